"""Every ou_conv tile shape x kernel variant (one tile per workgroup,
persistent, warp-specialised persistent; f32 and split-f16 operands) against a torch fp32
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
_KSWS = []


def _ksws():
    """K-slice workspace (64 MB, as an Engine holds)."""
    if not _KSWS:
        _KSWS.append(torch.empty(64 << 20 >> 2, dtype=torch.float32, device=DEV))
    return _KSWS[0]

# (cout, cin, frame, kt, T, batch, residual)
GEOMS = [
    (64, 64, 1, 3, 517, 2, False),
    (64, 64, 1, 5, 517, 2, True),
    (32, 32, 1, 3, 1000, 1, True),
    (96, 40, 1, 1, 77, 2, False),
    (512, 256, 1, 3, 33, 2, True),
    (64, 32, 2, 3, 300, 2, False),     # frame view, cin % chunk == 0 or not
    (48, 24, 5, 3, 203, 1, False),
    # more output tiles than CUs: persistent workgroups walk several tiles
    # (warp-specialised chunk stream across tile boundaries; split-K parity)
    (32, 32, 1, 3, 70000, 2, True),
    (256, 256, 1, 3, 3000, 2, True),
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
    cws = {0: E.make_conv(spec, DEV, prec=0), 1: E.make_conv(spec, DEV, prec=1)}
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
        # one-tile, persistent x2 / x4, warp-specialised; split-f16 (query bit 11)
        for v in (0, 1 << 8, 2 << 8, 1 << 10, 1 << 11):
            if not lib.ou_conv_tile_ok(kt, t | v):
                continue
            y = E.new_act(B, cout, U, DEV)
            ra = E.Act(res.to(DEV)) if with_res else None
            d = E.conv_desc(cws[1 if v == 1 << 11 else 0], xa, y, res1=ra, s1=0.7, n_frames=U)
            d.tile = t | (v & ~(1 << 11))
            rc = lib.ou_conv(ctypes.byref(d), ctypes.c_void_p(stream))
            if rc == -2 and v == 1 << 10:
                continue   # warp-specialised form refused for this geometry (single K chunk, rout > 1)
            assert rc == 0
            torch.cuda.synchronize()
            err = ((y.t.cpu() - ref).norm() / ref.norm()).item()
            if not err < 1e-5:
                bad.append((t, v, err))
        # K slices (two launches: partial sums, then reduce + epilogue), both precisions
        for prec, sl in ((0, 1), (1, 2), (1, 3)):
            if not lib.ou_conv_tile_ok(kt, t | (prec << 11)):
                continue
            y = E.new_act(B, cout, U, DEV)
            ra = E.Act(res.to(DEV)) if with_res else None
            d = E.conv_desc(cws[prec], xa, y, res1=ra, s1=0.7, n_frames=U)
            d.ks_ws, d.ks_ws_bytes = _ksws().data_ptr(), _ksws().numel() * 4
            d.tile = t | (sl << 12)
            rc = lib.ou_conv(ctypes.byref(d), ctypes.c_void_p(stream))
            if rc == -2:
                continue   # more K slices than chunks, or workspace too small
            assert rc == 0
            torch.cuda.synchronize()
            err = ((y.t.cpu() - ref).norm() / ref.norm()).item()
            if not err < 1e-5:
                bad.append((t, "ks", prec, sl, err))
    assert not bad, bad


@pytest.mark.parametrize("geom", [(96, 40, 1, 3, 301, 2), (64, 64, 1, 3, 40000, 2)], ids=str)
def test_conv_full_epilogue_every_tile(geom):
    """bias + residual 1 + FiLM + residual 2 + valid_len zeroing, every tile
    shape and kernel variant (ou_conv_desc formula, include/ouhip.h)."""
    cout, cin, frame, kt, T, B = geom
    g = torch.Generator().manual_seed(7)
    w = torch.randn(cout, cin * frame, kt, generator=g) * 0.1
    bias = torch.randn(cout, generator=g) * 0.1
    spec = E.ConvSpec(w.numpy(), cin, frame, (kt - 1) // 2, 1, 0.25, bias.numpy())
    cws = {0: E.make_conv(spec, DEV, prec=0), 1: E.make_conv(spec, DEV, prec=1)}
    x = torch.randn(B, cin, T, generator=g)
    U = -(-T // frame)
    r1 = torch.randn(B, cout, U, generator=g)
    r2 = torch.randn(B, cout, U, generator=g)
    film = torch.randn(B, 2 * cout, generator=g)
    valid = U - 3
    y0 = _ref(w, bias, x, frame, kt, 0.25, None, 1.0)
    y0[:, :, valid:] = 0.0
    ref = (y0 + r1) * 0.7
    ref = film[:, :cout, None] * ref + film[:, cout:, None]
    ref = (ref + r2) * 0.5
    xa, r1a, r2a = E.Act(x.to(DEV)), E.Act(r1.to(DEV)), E.Act(r2.to(DEV))
    fd = film.to(DEV)
    lib = L.load()
    stream = torch.cuda.current_stream().cuda_stream
    bad = []
    for t in range(lib.ou_conv_num_tiles()):
        for v in (0, 1 << 8, 2 << 8, 1 << 10, 1 << 11):
            if not lib.ou_conv_tile_ok(kt, t | v):
                continue
            y = E.new_act(B, cout, U, DEV)
            d = E.conv_desc(cws[1 if v == 1 << 11 else 0], xa, y, res1=r1a, s1=0.7, film=fd.data_ptr(),
                            film_bs=2 * cout, res2=r2a, s2=0.5, n_frames=U, valid_len=valid)
            d.tile = t | (v & ~(1 << 11))
            rc = lib.ou_conv(ctypes.byref(d), ctypes.c_void_p(stream))
            if rc == -2 and v == 1 << 10:
                continue   # warp-specialised form refused for this geometry (single K chunk, rout > 1)
            assert rc == 0
            torch.cuda.synchronize()
            err = ((y.t.cpu() - ref).norm() / ref.norm()).item()
            if not err < 1e-5:
                bad.append((t, v, err))
    assert not bad, bad


def test_split_range_flag():
    """split-f16: an input at or above 2^21 sets the status word (the host then
    reruns with f32 operands); inputs inside the range leave it clear and
    match the f32 form."""
    g = torch.Generator().manual_seed(5)
    cout, cin, kt, T = 64, 64, 3, 900
    w = torch.randn(cout, cin, kt, generator=g) * 0.1
    spec = E.ConvSpec(w.numpy(), cin, 1, 1, 1, 0.25, None)
    cw = E.make_conv(spec, DEV, prec=1)
    status = torch.zeros(4, dtype=torch.int32, device=DEV)
    stream = torch.cuda.current_stream().cuda_stream
    for scale, want in ((1.5e6, 0), (3.0e6, 1)):
        x = torch.randn(1, cin, T, generator=g)
        x[0, 5, 17] = scale
        y = E.new_act(1, cout, T, DEV)
        d = E.conv_desc(cw, E.Act(x.to(DEV)), y)
        d.status = status.data_ptr() + 4
        L.run_now(L.OP_CONV, d, stream)
        torch.cuda.synchronize()
        assert int(status[1]) == want, (scale, status.tolist())
        if want == 0:
            ref = _ref(w, None, x, 1, kt, 0.25, None, 1.0)
            assert ((y.t.cpu() - ref).norm() / ref.norm()).item() < 1e-5
        status.zero_()


@pytest.mark.parametrize("geom", GEOMS[:5], ids=[str(g) for g in GEOMS[:5]])
def test_conv_f16_every_tile(geom):
    """f16 operands (ConvDesc.prec = 2): every tile, alone and in 2 / 4 K
    slices, within f16 rounding of the f32 reference (operands rounded to 11
    bits, f32 accumulation)."""
    cout, cin, frame, kt, T, B, with_res = geom
    g = torch.Generator().manual_seed(hash(geom) % 1000)
    w = torch.randn(cout, cin * frame, kt, generator=g) * 0.1
    bias = torch.randn(cout, generator=g) * 0.1
    spec = E.ConvSpec(w.numpy(), cin, frame, (kt - 1) // 2, 1, 0.25, bias.numpy())
    cw = E.make_conv(spec, DEV, prec=2)
    x = torch.randn(B, cin, T, generator=g)
    U = -(-T // frame)
    ref = _ref(w, bias, x, frame, kt, 0.25, None, 1.0)
    xa = E.Act(x.to(DEV))
    lib = L.load()
    stream = torch.cuda.current_stream().cuda_stream
    ws = torch.empty(E.KSWS_BYTES // 4, dtype=torch.float32, device=DEV)   # K-slice partial sums
    bad, n = [], 0
    for t in range(lib.ou_conv_num_tiles()):
        if not lib.ou_conv_tile_ok(kt, t | (1 << 11)):
            continue
        for ks in (0, 1 << 12, 2 << 12):   # one workgroup per tile, 2 and 4 K slices
            y = E.new_act(B, cout, U, DEV)
            d = E.conv_desc(cw, xa, y, n_frames=U)
            d.ks_ws, d.ks_ws_bytes = ws.data_ptr(), E.KSWS_BYTES
            d.tile = t | ks
            rc = lib.ou_conv(ctypes.byref(d), ctypes.c_void_p(stream))
            if rc == -2 and ks:
                continue   # more K slices than K chunks
            assert rc == 0
            torch.cuda.synchronize()
            err = ((y.t.cpu() - ref).norm() / ref.norm()).item()
            n += 1
            if not (1e-5 < err < 2e-3):   # f16-rounded, not f32-exact, and not wrong
                bad.append((t, ks, err))
    assert n and not bad, bad


RS_BIT = 1 << 14
# (m, cin, frame, kt, rout, T, batch): deep same-convs, the GRU input
# projection, a transposed (rout) up-conv, frame-view (strided) down-convs
# with and without the folded FIR, rows past M and a ragged short clip
RS_GEOMS = [
    (512, 512, 1, 3, 1, 801, 1),
    (512, 512, 1, 5, 1, 203, 2),
    (256, 256, 1, 3, 1, 1001, 2),
    (1536, 512, 1, 1, 1, 99, 1),
    (1280, 512, 1, 3, 5, 157, 1),
    (96, 48, 1, 3, 1, 77, 2),
    (48, 80, 1, 1, 1, 45, 1),
    (128, 64, 4, 3, 1, 2003, 2),
    (64, 32, 2, 1, 1, 999, 1),
    (256, 128, 4, 3, 1, 401, 1),
    # K chunked through LDS: the conditioner's st_convs (rates 160 / 20),
    # the rate-5 down conv, a frame-1 conv over 2048 channels
    (512, 32, 160, 1, 1, 6401, 1),
    (512, 128, 20, 1, 1, 2001, 2),
    (512, 256, 5, 3, 1, 1003, 1),
    (64, 2048, 1, 1, 1, 100, 1),
    # fewer K steps than K-split waves (16 channels x 1 tap: one step)
    (32, 16, 1, 1, 2, 440, 2),
    (32, 16, 1, 3, 1, 300, 1),
]


@pytest.mark.parametrize("geom", RS_GEOMS, ids=[str(g) for g in RS_GEOMS])
def test_conv_register_streamed_every_shape(geom):
    """The register-streamed kernel (tile bit 14), every shape, split-f16 and
    f16, with the full epilogue (bias, residual 1, FiLM, residual 2, valid_len,
    the rout pixel shuffle, the frame view): equal to the chunked kernel on the
    same packed weights up to f32 summation order."""
    m, cin, frame, kt, rout, T, B = geom
    g = torch.Generator().manual_seed(m + cin + kt + frame)
    w = torch.randn(m, cin * frame, kt, generator=g) * (1.0 / np.sqrt(cin * frame * kt))
    cout = m // rout
    bias = torch.randn(cout, generator=g) * 0.1
    spec = E.ConvSpec(w.numpy(), cin, frame, (kt - 1) // 2, rout, 0.25, bias.numpy())
    x = torch.randn(B, cin, T, generator=g)
    U = -(-T // frame)
    L_out = U * rout
    r1 = torch.randn(B, cout, L_out, generator=g)
    r2 = torch.randn(B, cout, L_out, generator=g)
    film = torch.randn(B, 2 * cout, generator=g).to(DEV)
    xa, r1a, r2a = E.Act(x.to(DEV)), E.Act(r1.to(DEV)), E.Act(r2.to(DEV))
    lib = L.load()
    stream = torch.cuda.current_stream().cuda_stream
    ws = torch.empty(E.KSWS_BYTES // 4, dtype=torch.float32, device=DEV)   # K-slice partial sums
    bad, n, nks = [], 0, 0
    for prec in (1, 2):
        cw = E.make_conv(spec, DEV, prec=prec)

        def run(tile):
            y = E.new_act(B, cout, L_out, DEV)
            d = E.conv_desc(cw, xa, y, res1=r1a, s1=0.7, film=film.data_ptr(), film_bs=2 * cout, res2=r2a,
                            s2=0.5, n_frames=U, out_len=L_out, valid_len=L_out - 2)
            d.tile = tile
            d.ks_ws, d.ks_ws_bytes = ws.data_ptr(), E.KSWS_BYTES
            rc = lib.ou_conv(ctypes.byref(d), ctypes.c_void_p(stream))
            torch.cuda.synchronize()
            return rc, y.t.cpu()

        rc, ref = run(-1)
        assert rc == 0
        if prec == 1 and rout == 1:   # the chunked kernel itself against torch fp32
            want = _ref(w, bias, x, frame, kt, 0.25, None, 1.0)
            want[:, :, L_out - 2:] = 0.0
            want = film.cpu()[:, :cout, None] * ((want + r1) * 0.7) + film.cpu()[:, cout:, None]
            want = (want + r2) * 0.5
            assert ((ref - want).norm() / want.norm()).item() < 1e-5
        for t in range(16):
            if not lib.ou_conv_tile_ok(kt, t | RS_BIT):
                continue
            rc, y = run(t | RS_BIT)
            if rc == -2:
                continue   # input window over LDS for this shape
            assert rc == 0, lib.ou_last_error()
            n += 1
            err = ((y - ref).norm() / ref.norm()).item()
            if not err < 2e-6:
                bad.append((prec, t, err))
            # K slices (K-chunked windows only; refused where chunks < slices)
            for k in (1, 2, 3):
                rc, y = run(t | RS_BIT | (k << 12))
                if rc == -2:
                    continue
                assert rc == 0, lib.ou_last_error()
                nks += 1
                err = ((y - ref).norm() / ref.norm()).item()
                if not err < 2e-6:
                    bad.append((prec, t, 1 << k, err))
    assert n >= 6 and not bad, bad
    if cin * frame >= 2048 and frame > 1:   # the st_conv shapes: K-chunked, so sliceable
        assert nks > 0
