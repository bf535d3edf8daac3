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
    "ou_ensemble_args": L.EnsembleArgs, "ou_block_desc": L.BlockDesc, "ou_sync_args": L.SyncArgs,
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
    """Packed order: [mtile][pair // 4][tap][lane][pair % 4], lane -> (row =
    lane & 31, channel = 2 * pair + (lane >> 5)); channels zero-padded to a
    multiple of 64 (one float4 per lane = 4 consecutive k-steps)."""
    rng = np.random.default_rng(0)
    m, cin, kt = 40, 20, 3
    w = rng.standard_normal((m, cin, kt)).astype(np.float32)
    packed = L.conv_pack(w, L.conv_chunk(kt, 1))
    mtiles, pairs = 2, 32
    ref = np.zeros((mtiles, pairs // 4, kt, 64, 4), np.float32)
    for mt in range(mtiles):
        for cp in range(pairs):
            for k in range(kt):
                for lane in range(64):
                    row, c = mt * 32 + (lane & 31), 2 * cp + (lane >> 5)
                    if row < m and c < cin:
                        ref[mt, cp // 4, k, lane, cp % 4] = w[row, c, k]
    np.testing.assert_array_equal(packed, ref.reshape(-1))


def test_conv_tiles_fit_lds():
    lib = L.load()
    n = lib.ou_conv_num_tiles()
    assert n >= 6
    for kt in (1, 3, 4, 5):
        assert any(lib.ou_conv_tile_ok(kt, t) for t in range(n))


def test_conv_pack_split_layout():
    """Split-f16 order [mtile][pair // 8][hi | lo][tap][lane][pair % 8] of
    a = w * 2^e (max|a| in [2^9, 2^10)): hi + lo * 2^-11 restores a to ~2^-22;
    w_unscale = 2^(6 - e) (the kernel stages its input as x * 2^-6)."""
    rng = np.random.default_rng(1)
    m, cin, kt = 40, 20, 3
    w = (rng.standard_normal((m, cin, kt)) * 0.03).astype(np.float32)
    packed, unscale = L.conv_pack_split(w)
    assert packed.size == L.load().ou_conv_packed_size(m, cin, kt, 0)
    e = 6 - int(np.log2(unscale))
    assert 2.0**9 <= np.abs(w).max() * 2.0**e < 2.0**10
    h = packed.view(np.float16).astype(np.float64).reshape(2, 64 // 16, 2, kt, 64, 8)
    a = h[:, :, 0] + h[:, :, 1] / 2048.0
    ref = np.zeros((2, 4, kt, 64, 8))
    for mt in range(2):
        for g in range(4):
            for k in range(kt):
                for lane in range(64):
                    for j in range(8):
                        row, c = mt * 32 + (lane & 31), 2 * (8 * g + j) + (lane >> 5)
                        if row < m and c < cin:
                            ref[mt, g, k, lane, j] = float(w[row, c, k]) * 2.0**e
    assert np.abs(a - ref).max() <= 2.0**-21 * np.abs(ref).max()
    assert np.count_nonzero(ref) == np.count_nonzero(h[:, :, 0])


@pytest.mark.parametrize("field", ["x", "y", "res1"])
def test_conv_rejects_per_item_tensors_past_the_buffer_range(field):
    """Kernels address a batch item through a 32-bit buffer resource with a
    sentinel offset for "outside": ou_conv refuses a per-item tensor that
    reaches the sentinel (host-side validation, refused before any HIP call)."""
    lib = L.load()
    d = L.ConvDesc()
    d.x = d.w = d.y = 256
    d.m, d.cin, d.kt, d.frame, d.rout, d.batch = 64, 64, 3, 1, 1, 1
    d.n_frames = d.in_len = d.out_len = 1000
    d.x_cstride = d.y_cstride = d.r1_cstride = 1000
    big = (1 << 31) // (4 * 64)   # 64 channels x big floats = 2 GiB
    if field == "res1":
        d.res1 = 256
    setattr(d, f"{'r1' if field == 'res1' else field}_cstride", big)
    assert lib.ou_conv(ctypes.byref(d), None) == -1
    assert b"32-bit buffer range" in lib.ou_last_error()


@pytest.mark.parametrize("field", ["h", "y", "sc", "co"])
def test_block_rejects_per_item_tensors_past_the_buffer_range(field):
    lib = L.load()
    d = L.BlockDesc()
    d.h = d.y = d.w[0] = d.w[1] = d.w[2] = 256
    d.channels, d.length, d.batch, d.prec = 64, 1000, 1, 1
    d.h_cstride = d.y_cstride = d.sc_cstride = d.co_cstride = 1000
    if field == "sc":
        d.sc = 256
    if field == "co":
        d.cond_out = 256
    setattr(d, f"{field}_cstride", (1 << 31) // (4 * 64))
    assert lib.ou_block(ctypes.byref(d), None) == -1
    assert b"32-bit buffer range" in lib.ou_last_error()
