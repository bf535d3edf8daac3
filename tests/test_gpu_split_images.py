"""Split images on the GPU (include/ouhip.h, ou_conv_desc.sy / xs): the
split-image kernel (tile bit 15) against a torch fp32 reference of the same
convolution for every shape (plain / frame view / 1x1 / transposed,
ragged lengths, batch 2, residual epilogue), the split image a producer's
epilogue stores against its restatement, and the per-layer staging exponent
with its range codes (1: a staged input, 2: a stored split image, 4:
infinite)."""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from open_universe_amd import _lib as L
from open_universe_amd import engine as E

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def split_image(x, slope, shift, rows=None):
    """prelu(x) * 2^-shift as [B][C / 32][rows][hi | lo][32] f16 (int16 view)."""
    B, C, T = x.shape
    rows = T if rows is None else rows
    p = x.float() * 2.0 ** -shift
    p = torch.where(p >= 0, p, p * slope)
    hi = p.half()
    lo = ((p - hi.float()) * 2048.0).half()
    img = torch.zeros(B, C // 32, rows, 2, 32, dtype=torch.float16, device=x.device)
    img[:, :, :T, 0, :] = hi.reshape(B, C // 32, 32, T).transpose(2, 3)
    img[:, :, :T, 1, :] = lo.reshape(B, C // 32, 32, T).transpose(2, 3)
    return img.view(torch.int16).reshape(-1)


def image_values(img, B, C, T, rows):
    v = img.view(torch.float16).reshape(B, C // 32, rows, 2, 32).double()
    val = v[:, :, :T, 0, :] + v[:, :, :T, 1, :] / 2048.0
    return val.transpose(2, 3).reshape(B, C, T)


def _ref(w, b, x, frame, kt, slope, res, s1, rout=1):
    B, cin, T = x.shape
    U = -(-T // frame)
    xp = F.pad(x, (0, U * frame - T))
    xv = xp.reshape(B, cin, U, frame).permute(0, 1, 3, 2).reshape(B, cin * frame, U)
    xv = torch.where(xv >= 0, xv, xv * slope)
    y = F.conv1d(xv.double(), w.double(), b.double(), padding=(kt - 1) // 2)
    if rout > 1:   # channel-major rows m = co * rout + ph -> sample u * rout + ph
        y = y.reshape(B, -1, rout, U).permute(0, 1, 3, 2).reshape(B, -1, U * rout)
    if res is not None:
        y = (y + res.double()) * s1
    return y


# (cout, cin, frame, kt, T, batch, residual, rout)
GEOMS = [
    (512, 512, 1, 3, 801, 1, True, 1),      # the 512-channel level at C2
    (512, 512, 1, 5, 801, 1, False, 1),
    (256, 256, 1, 3, 4005, 1, True, 1),     # the 256-channel level
    (1536, 512, 1, 1, 801, 1, False, 1),    # GRU input projection
    (512, 256, 5, 3, 4005, 1, False, 1),    # down conv, rate 5 (frame view)
    (256, 128, 4, 3, 16020, 1, False, 1),   # down conv, rate 4
    (256, 512, 1, 3, 801, 1, True, 5),      # up conv, rate 5 (channel-major rows)
    (64, 96, 1, 3, 333, 2, True, 1),        # batch 2, ragged, 3 chunks over 4 waves
    (32, 32, 1, 5, 77, 2, False, 1),        # one chunk: three waves run zero chunks
]


@pytest.mark.parametrize("geom", GEOMS, ids=[str(g) for g in GEOMS])
def test_split_image_kernel_every_shape(geom):
    cout, cin, frame, kt, T, B, with_res, rout = geom
    g = torch.Generator().manual_seed(sum(geom))
    m = cout * rout
    w = torch.randn(m, cin * frame, kt, generator=g) * 0.05
    bias = torch.randn(cout, generator=g) * 0.1
    spec = E.ConvSpec(w.numpy(), cin, frame, (kt - 1) // 2, rout, 0.25,
                      np.repeat(bias.numpy(), 1), cm=rout > 1)
    cw = E.make_conv(spec, DEV, prec=1)
    assert cw.w_nat is not None
    x = torch.randn(B, cin, T, generator=g)
    U = -(-T // frame)
    res = torch.randn(B, cout, U * rout, generator=g) if with_res else None
    # the kernel's weight rows for rout > 1 are channel-major (m = co * rout + ph): bias per channel
    ref = _ref(w, bias.repeat_interleave(rout) if rout > 1 else bias, x, frame, kt, 0.25, res, 0.7, rout)
    xa = E.Act(x.to(DEV))
    img = split_image(xa.t, 0.25, 6, rows=T + 2)
    lib = L.load()
    stream = torch.cuda.current_stream().cuda_stream
    for shape in range(6):
        for mj in (0, 1 << 16):
            y = E.new_act(B, cout, U * rout, DEV)
            y.t.fill_(float("nan"))
            ra = E.Act(res.to(DEV)) if with_res else None
            d = E.conv_desc(cw, xa, y, res1=ra, s1=0.7, n_frames=U)
            d.xs, d.xs_bstride, d.xs_rows, d.xs_shift = img.data_ptr(), img.numel() * 2 // B, T + 2, 6
            d.w, d.w_unscale = cw.w_nat.data_ptr(), cw.w_unscale_nat
            d.tile = L.SS_BIT | shape | mj
            assert lib.ou_conv(ctypes.byref(d), ctypes.c_void_p(stream)) == 0, lib.ou_last_error()
            torch.cuda.synchronize()
            err = ((y.t.cpu().double() - ref).norm() / ref.norm()).item()
            assert err < 1e-5, (shape, mj, err)


@pytest.mark.parametrize("tile", [11, 11 | (1 << 12), E.RS_BIT | 2, L.SS_BIT | 1])
def test_producer_stores_split_image(tile):
    """A conv with ou_conv_desc.sy stores prelu_{a'}(y) 2^-s beside y (the
    chunked, K-sliced, register-streamed and split-image kernels alike)."""
    C, T, B = 256, 1003, 2
    g = torch.Generator().manual_seed(tile & 0xffff)
    w = torch.randn(C, C, 3, generator=g) * 0.05
    spec = E.ConvSpec(w.numpy(), C, 1, 1, 1, 0.25, np.zeros(C, np.float32))
    cw = E.make_conv(spec, DEV, prec=1)
    x = E.Act(torch.randn(B, C, T, device=DEV))
    y = E.new_act(B, C, T, DEV)
    rows = T + 5
    sy = torch.full((B * (C // 32) * rows * 64,), 0x7e00, dtype=torch.int16, device=DEV)
    d = E.conv_desc(cw, x, y)
    ws = torch.empty(E.KSWS_BYTES // 4, dtype=torch.float32, device=DEV)   # K-slice partial sums
    d.ks_ws, d.ks_ws_bytes = ws.data_ptr(), E.KSWS_BYTES
    if tile & L.SS_BIT:
        img = split_image(x.t, 0.25, 6)
        d.xs, d.xs_bstride, d.xs_rows, d.xs_shift = img.data_ptr(), img.numel() * 2 // B, T, 6
        d.w, d.w_unscale = cw.w_nat.data_ptr(), cw.w_unscale_nat
    d.sy, d.sy_bstride, d.sy_rows, d.sy_shift, d.sy_slope = sy.data_ptr(), (C // 32) * rows * 128, rows, 9, 0.125
    d.tile = tile
    assert L.load().ou_conv(ctypes.byref(d), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    torch.cuda.synchronize()
    p = y.t.double() * 2.0 ** -9
    p = torch.where(p >= 0, p, p * 0.125)
    got = image_values(sy, B, C, T, rows)
    assert ((got - p).abs() <= p.abs() * 2.0 ** -21 + 2.0 ** -35).all()
    tail = sy.view(B, C // 32, rows, 64)[:, :, T:]
    assert (tail == 0x7e00).all()   # rows past out_len never written


def test_staging_exponent_and_range_codes():
    """xs_shift widens a conv's split-f16 range: inputs of 2^22 overflow at
    the default 2^-6 (range code 1 in the conv's status word; a producer
    storing them as a split image: code 2) and are exact at 2^-10."""
    C, T = 128, 517
    g = torch.Generator().manual_seed(5)
    w = torch.randn(C, C, 3, generator=g) * 0.05
    spec = E.ConvSpec(w.numpy(), C, 1, 1, 1, 0.25, np.zeros(C, np.float32))
    cw = E.make_conv(spec, DEV, prec=1)
    x = torch.randn(1, C, T, generator=g) * 2.0 ** 22
    ref = _ref(w, torch.zeros(C), x, 1, 3, 0.25, None, 1.0)
    xa, y = E.Act(x.to(DEV)), E.new_act(1, C, T, DEV)
    st = torch.zeros(4, dtype=torch.int32, device=DEV)
    lib = L.load()
    stream = torch.cuda.current_stream().cuda_stream
    for shift, tile in ((6, 11), (10, 11), (6, E.RS_BIT | 2), (10, E.RS_BIT | 2)):
        st.zero_()
        d = E.conv_desc(cw, xa, y)
        d.status, d.xs_shift, d.tile = st.data_ptr(), shift, tile
        assert lib.ou_conv(ctypes.byref(d), ctypes.c_void_p(stream)) == 0
        torch.cuda.synchronize()
        if shift == 6:
            assert st[0].item() == 1, (tile, st.tolist())
        else:
            assert st[0].item() == 0
            err = ((y.t.cpu().double() - ref).norm() / ref.norm()).item()
            assert err < 1e-5, (tile, err)
    # a producer storing a split image of values 2^22 at exponent 6: code 2
    st.zero_()
    sy = torch.zeros(C // 32 * T * 64, dtype=torch.int16, device=DEV)
    d = E.conv_desc(cw, xa, y)
    d.status, d.xs_shift, d.tile = st.data_ptr(), 10, 11
    d.sy, d.sy_bstride, d.sy_rows, d.sy_shift, d.sy_slope = sy.data_ptr(), C // 32 * T * 128, T, 6, 1.0
    assert lib.ou_conv(ctypes.byref(d), ctypes.c_void_p(stream)) == 0
    torch.cuda.synchronize()
    assert st[0].item() == 2, st.tolist()


def test_fused_block_split_image_links():
    """Split images through a fused block (ou_block_desc.xs / sy): conv ->
    block -> conv recorded with the split-image hook links the block to both
    neighbours (it reads the first conv's image at stage 0 and stores the
    last conv's operand), and the result equals the unlinked program's and a
    float64 evaluation."""
    from test_gpu_block import _ref as block_ref, _specs

    C, T, B = 128, 1003, 2
    g = torch.Generator().manual_seed(11)
    specs = _specs(C, g)
    cws = [E.make_conv(sp, DEV, prec=1) for sp in specs]
    bw = E.BlockW(C, "none", None, *cws, None, E.prep_fused(specs, C, 1, DEV))
    wa, wb = (torch.randn(C, C, 3, generator=g) * 0.05 for _ in range(2))
    ca, cb = (E.make_conv(E.ConvSpec(w.numpy(), C, 1, 1, 1, 0.2, np.zeros(C, np.float32)), DEV, prec=1)
              for w in (wa, wb))
    x = torch.randn(B, C, T, generator=g)
    h_ref = _ref(wa, torch.zeros(C), x, 1, 3, 0.2, None, 1.0)
    y_ref, _ = block_ref(specs, h_ref)
    z_ref = _ref(wb, torch.zeros(C), y_ref, 1, 3, 0.2, None, 1.0)
    xa = E.Act(x.to(DEV))
    outs = {}
    saved = L.ADD_HOOK
    try:
        for linked in (False, True):
            E.begin_record(1 if linked else 0, DEV)
            prog = L.Program()
            h, y, z = (E.new_act(B, C, T, DEV) for _ in range(3))
            tA, tB = E.new_act(B, C, T, DEV), E.new_act(B, C, T, DEV)
            prog.add(L.OP_CONV, E.conv_desc(ca, xa, h))
            E.rec_block(prog, bw, h, y, tA, tB)
            prog.add(L.OP_CONV, E.conv_desc(cb, y, z))
            E.end_record()
            links = getattr(prog, "split_links", [])
            assert len(links) == (2 if linked else 0), links
            prog.run(torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            outs[linked] = (y.t.cpu().double(), z.t.cpu().double())
    finally:
        E.end_record()
        L.ADD_HOOK = saved
    for k in (0, 1):
        a, b = outs[True][k], outs[False][k]
        assert ((a - b).norm() / b.norm()).item() < 1e-6
    assert ((outs[True][0] - y_ref).norm() / y_ref.norm()).item() < 1e-5
    assert ((outs[True][1] - z_ref).norm() / z_ref.norm()).item() < 1e-5
