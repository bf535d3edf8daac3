"""Every ou_conv tile shape x tiles-per-workgroup against a torch fp32
reference of the same convolution (ragged lengths, batch 2, residual epilogue,
frame view).  A tile the autotuner might pick must be exact up to fp32
summation order."""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from open_universe_amd import _lib as L
from open_universe_amd import engine as E

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

# (cout, cin, frame, kt, T, batch, residual)
GEOMS = [
    (64, 64, 1, 3, 517, 2, False),
    (64, 64, 1, 5, 517, 2, True),
    (32, 32, 1, 3, 1000, 1, True),
    (96, 40, 1, 1, 77, 2, False),
    (512, 256, 1, 3, 33, 2, True),
    (64, 32, 2, 3, 300, 2, False),     # frame view, cin % chunk == 0 or not
    (48, 24, 5, 3, 203, 1, False),
]


def _ref(w, b, x, frame, kt, slope, res, s1):
    # frame view (logical channel ci*R + ph) as a strided reshape of x
    B, cin, T = x.shape
    U = -(-T // frame)
    xp = F.pad(x, (0, U * frame - T))
    xv = xp.reshape(B, cin, U, frame).permute(0, 1, 3, 2).reshape(B, cin * frame, U)
    xv = torch.where(xv >= 0, xv, xv * slope)
    y = F.conv1d(xv, w, b, padding=(kt - 1) // 2)
    if res is not None:
        y = (y + res) * s1
    return y


@pytest.mark.parametrize("geom", GEOMS, ids=[str(g) for g in GEOMS])
def test_conv_every_tile(geom):
    cout, cin, frame, kt, T, B, with_res = geom
    g = torch.Generator().manual_seed(hash(geom) % 1000)
    w = torch.randn(cout, cin * frame, kt, generator=g) * 0.1
    bias = torch.randn(cout, generator=g) * 0.1
    spec = E.ConvSpec(w.numpy(), cin, frame, (kt - 1) // 2, 1, 0.25, bias.numpy())
    cw = E.make_conv(spec, DEV)
    x = torch.randn(B, cin, T, generator=g)
    U = -(-T // frame)
    res = torch.randn(B, cout, U, generator=g) if with_res else None
    ref = _ref(w, bias, x, frame, kt, 0.25, res, 0.7)
    xa = E.Act(x.to(DEV))
    lib = L.load()
    stream = torch.cuda.current_stream().cuda_stream
    bad = []
    for t in range(lib.ou_conv_num_tiles()):
        if not lib.ou_conv_tile_ok(kt, t):
            continue
        for tpw in (0, 1, 2):
            if not lib.ou_conv_tile_ok(kt, t | (tpw << 8)):
                continue
            y = E.new_act(B, cout, U, DEV)
            ra = E.Act(res.to(DEV)) if with_res else None
            d = E.conv_desc(cw, xa, y, res1=ra, s1=0.7, n_frames=U)
            d.tile = t | (tpw << 8)
            assert lib.ou_conv(ctypes.byref(d), ctypes.c_void_p(stream)) == 0
            torch.cuda.synchronize()
            err = ((y.t.cpu() - ref).norm() / ref.norm()).item()
            if not err < 1e-5:
                bad.append((t, tpw, err))
    assert not bad, bad
