"""The C-ABI library: loads, exports every symbol include/ouhip.h declares, and
the ctypes mirrors of the descriptor structs have the C compiler's layout.
(No compute calls: runs without a GPU.)"""
import ctypes
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

from open_universe_amd import _lib as L

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "ouhip.h")


def test_library_loads_and_version():
    lib = L.load()
    assert lib.ou_abi_version() == L.ABI_VERSION


def test_every_declared_symbol_is_exported():
    text = open(HEADER).read()
    declared = set(re.findall(r"\b(ou_[a-z0-9_]+)\s*\(", text))
    declared -= {"ou_program"}
    lib = ctypes.CDLL(L.LIB_PATH)
    missing = [s for s in sorted(declared) if not hasattr(lib, s)]
    assert not missing, missing
    assert declared == set(L.EXPORTS), declared ^ set(L.EXPORTS)


STRUCTS = {
    "ou_conv_desc": L.ConvDesc, "ou_gru_desc": L.GruDesc, "ou_embed_desc": L.EmbedDesc,
    "ou_head_desc": L.HeadDesc, "ou_snake_desc": L.SnakeDesc, "ou_memset_desc": L.MemsetArgs,
    "ou_norm_args": L.NormArgs, "ou_rms_args": L.RmsArgs, "ou_power_args": L.PowerArgs,
    "ou_pad_args": L.PadArgs, "ou_scale_args": L.ScaleArgs, "ou_finish_args": L.FinishArgs,
    "ou_ensemble_args": L.EnsembleArgs,
}


def test_struct_layouts_match_c():
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void){"]
    for cname, py in STRUCTS.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'printf("{cname}.{fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0;}")
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "l.c"), os.path.join(d, "l")
        open(src, "w").write("\n".join(lines))
        subprocess.check_call(["gcc", "-std=c99", "-o", exe, src])
        out = subprocess.check_output([exe]).decode().split("\n")
    got = dict(line.rsplit(" ", 1) for line in out if line)
    for cname, py in STRUCTS.items():
        assert int(got[f"{cname} size"]) == ctypes.sizeof(py), cname
        for fname, _ in py._fields_:
            assert int(got[f"{cname}.{fname}"]) == getattr(py, fname).offset, (cname, fname)


def test_conv_pack_layout():
    """Packed order: [mtile][chunk][cp][k][lane], lane -> (row = lane & 31,
    channel = chunk*cc + cp + (lane >> 5) * cc/2), zero padded."""
    rng = np.random.default_rng(0)
    m, cin, kt = 40, 20, 3
    w = rng.standard_normal((m, cin, kt)).astype(np.float32)
    cc = L.conv_chunk(kt, 1)
    packed = L.conv_pack(w, cc)
    mtiles, nch, half = 2, -(-cin // cc), cc // 2
    ref = np.zeros((mtiles, nch, half, kt, 64), np.float32)
    for mt in range(mtiles):
        for q in range(nch):
            for cp in range(half):
                for k in range(kt):
                    for lane in range(64):
                        row, c = mt * 32 + (lane & 31), q * cc + cp + (lane >> 5) * half
                        if row < m and c < cin:
                            ref[mt, q, cp, k, lane] = w[row, c, k]
    np.testing.assert_array_equal(packed, ref.reshape(-1))


@pytest.mark.parametrize("kt,frame,cc", [(5, 1, 16), (3, 1, 16), (1, 1, 32), (3, 5, 40),
                                         (1, 160, 160), (4, 160, 160), (3, 3, 24), (1, 20, 40)])
def test_conv_chunk(kt, frame, cc):
    assert L.conv_chunk(kt, frame) == cc
