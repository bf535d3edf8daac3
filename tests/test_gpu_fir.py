"""The FIR-applied rate-change kernels (tile bit 17, ou_conv_desc.fir:
conv_fdkernel / conv_fukernel) on the GPU, through the C ABI.

PReLU_Conv with use_antialiasing (reference networks/universe/blocks.py:214-226)
runs the binomial FIR (blocks.py:66-72, 123-134) before a strided conv or after
a transposed one.  Every FIR tile shape, both directions, every rate the
configs use (2, 3, 4, 5, 8), split-f16 and f16 operands, against a float64
torch evaluation of the reference's op sequence; and the FIR-applied form
against the folded form (engine.spec_down / spec_up) of the same layer.
Tolerances: split-f16 rel-RMS <= 1e-5 (f32 class), f16 <= 3e-3."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import rel_rms
from open_universe_amd import _lib as L
from open_universe_amd import dsp
from open_universe_amd import engine as E

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _sd(direction, cin, cout, r, seed):
    """A plain (no weight norm) PReLU_Conv state dict with a bias."""
    g = torch.Generator().manual_seed(seed)
    shape = (cout, cin, r) if direction == "down" else (cin, cout, r)
    return {"p.conv.weight": torch.randn(shape, generator=g) * 0.2,
            "p.prelu.weight": torch.tensor([0.25]),
            "p.bias": torch.randn(cout, generator=g)}


def _ref(sd, direction, r, x, res=None, s1=1.0):
    """blocks.py:214-231 in float64: prelu -> FIR -> strided conv (down), or
    prelu -> transposed conv -> FIR (up), then the bias; (+ res) * s1."""
    x = x.double()
    w = sd["p.conv.weight"].double()
    taps = torch.from_numpy(dsp.binomial_taps(2 * r + 1)).double()
    C = x.shape[1]
    x = torch.where(x >= 0, x, x * 0.25)
    fir = lambda v: F.conv1d(v, taps[None, None].expand(v.shape[1], 1, -1), padding="same", groups=v.shape[1])
    if direction == "down":
        T = x.shape[-1]
        x = F.pad(x, (0, (-T) % r))
        y = F.conv1d(fir(x), w, stride=r)
    else:
        y = fir(F.conv_transpose1d(x, w, stride=r))
    y = y + sd["p.bias"].double()[None, :, None]
    if res is not None:
        y = (y + res.double()) * s1
    return y


def _launch(d):
    L.run_now(L.OP_CONV, d, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()


def _case(direction, r, cin, cout, T, B, prec):
    sd = _sd(direction, cin, cout, r, seed=r * 10 + cin)
    spec = E.spec_down(sd, "p", r, True) if direction == "down" else E.spec_up(sd, "p", r, True)
    assert spec.fir is not None
    cw = E.make_conv(spec, DEV, prec=prec)
    x = torch.randn(B, cin, T, generator=torch.Generator().manual_seed(5))
    xa = E.Act(x.to(DEV))
    if direction == "down":
        U = -(-T // r)
        y = E.new_act(B, cout, U, DEV)
        d = E.conv_desc(cw, xa, y)
        res = None
        ref = _ref(sd, direction, r, x)
    else:
        res = torch.randn(B, cout, r * T, generator=torch.Generator().manual_seed(6))
        y = E.new_act(B, cout, r * T, DEV)
        d = E.conv_desc(cw, xa, y, n_frames=T, valid_len=r * T, res1=E.Act(res.to(DEV)), s1=float(E.NF2))
        ref = _ref(sd, direction, r, x, res, float(E.NF2))
    return d, y, ref


@pytest.mark.parametrize("prec", [1, 2])
@pytest.mark.parametrize("r", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("direction", ["down", "up"])
def test_fir_every_tile(direction, r, prec):
    cin, cout = (32, 64) if direction == "down" else (64, 32)
    d, y, ref = _case(direction, r, cin, cout, 301, 2, prec)
    f = E.fir_desc(d)
    lib = L.load()
    n = 0
    # up: early epilogue loads / two chunks in flight; down (bias only here): two chunks in flight
    early = (0, E.FIR_EARLY, E.FIR_DEEP) if direction == "up" else (0, E.FIR_DEEP)
    for shape in range(16):
        for mm in [m | e for m in (0, L.MAJ_BIT) for e in early]:
            t = E.FIR_BIT | shape | mm
            if not lib.ou_conv_tile_ok(1, t):
                continue
            y.t.fill_(float("nan"))
            f.tile = t
            _launch(f)
            err = rel_rms(y.t.cpu(), ref)
            assert err < (1e-5 if prec == 1 else 3e-3), (shape, mm, err)
            n += 1
    assert n >= 16


@pytest.mark.parametrize("direction,r,cin,cout,T,B", [
    ("down", 2, 48, 96, 2403, 3),      # PP24 score level 0
    ("down", 8, 384, 768, 1001, 2),    # PP24 level 3 (the deepest, K = 3072)
    ("down", 5, 256, 512, 803, 1),     # PP16 level 3
    ("up", 3, 192, 96, 1335, 2),       # PP24 decoder, rate 3 (whole channels: 10 per m-tile)
    ("up", 8, 768, 384, 1001, 2),      # PP24 decoder, rate 8
    ("up", 2, 64, 32, 4000, 1),        # PP16 decoder top level
])
def test_fir_matches_folded_form(direction, r, cin, cout, T, B):
    """The same layer in its two forms (folded 3-frame weights, tuned tile;
    FIR applied, default tile) against the float64 reference."""
    d, y, ref = _case(direction, r, cin, cout, T, B, 1)
    _launch(d)
    folded = y.t.cpu().clone()
    y.t.fill_(float("nan"))
    _launch(E.fir_desc(d))
    fir = y.t.cpu()
    assert rel_rms(folded, ref) < 1e-5
    assert rel_rms(fir, ref) < 1e-5


def test_fir_range_flag():
    """A staged FIR output of 2^15 or more (after the 2^-s staging scale)
    sets range code 1 in the status word."""
    d, y, ref = _case("down", 4, 32, 64, 257, 1, 1)
    st = torch.zeros(1, dtype=torch.int32, device=DEV)
    f = E.fir_desc(d)
    f.status = st.data_ptr()
    f.xs_shift = -16   # stage x 2^16: |FIR(prelu(x))| ~ 1 -> well past 2^15
    _launch(f)
    assert int(st.item()) & 1


@pytest.mark.parametrize("rt,cin,cout", [
    (240, 48, 768), (120, 96, 768), (40, 192, 768),    # PP24's st_convs (condition.py:53-59)
    (160, 32, 512), (80, 64, 512), (20, 128, 512),     # PP16's
])
def test_st_conv_fir3_every_tile(rt, cin, cout):
    """The conditioner's wide strided convs on the FIR down kernel without a
    FIR (ou_conv_desc.fir 3, K in chunks of 16 channels x 8 / 4 phases), every
    tile shape, in both epilogues: bias only (the lean one) and the st_conv
    running sum's two residuals, against float64 (ragged length: the last
    frame is zero-padded, as F.conv1d over the padded input)."""
    g = torch.Generator().manual_seed(rt + cin)
    sd = {"p.conv.weight": torch.randn(cout, cin, rt, generator=g) / np.sqrt(cin * rt),
          "p.prelu.weight": torch.tensor([0.25]), "p.conv.bias": torch.randn(cout, generator=g)}
    spec = E.spec_down(sd, "p", rt, False)
    assert spec.fir is not None and spec.fir[0] == 3
    cw = E.make_conv(spec, DEV, prec=1)
    B, U = 2, 37
    T = U * rt - 5
    x = torch.randn(B, cin, T, generator=g)
    r1, r2 = torch.randn(B, cout, U, generator=g), torch.randn(B, cout, U, generator=g)
    xd = torch.where(x.double() >= 0, x.double(), 0.25 * x.double())
    base = F.conv1d(F.pad(xd, (0, U * rt - T)), sd["p.conv.weight"].double(), stride=rt)
    base = base + sd["p.conv.bias"].double()[None, :, None]
    lib = L.load()
    n = 0
    for res in (False, True):
        y = E.new_act(B, cout, U, DEV)
        if res:
            d = E.conv_desc(cw, E.Act(x.to(DEV)), y, res1=E.Act(r1.to(DEV)), s1=1.0,
                            res2=E.Act(r2.to(DEV)), s2=0.5)
            ref = (base + r1.double() + r2.double()) * 0.5
        else:
            d = E.conv_desc(cw, E.Act(x.to(DEV)), y)
            ref = base
        f = E.fir_desc(d)
        assert f.fir == 3
        for shape in range(16):
            for mm in (0, L.MAJ_BIT):
                t = E.FIR_BIT | shape | mm
                if not lib.ou_conv_tile_ok(1, t):
                    continue
                y.t.fill_(float("nan"))
                f.tile = t
                _launch(f)
                err = rel_rms(y.t.cpu(), ref)
                assert err < 1e-5, (res, shape, mm, err)
                n += 1
    assert n >= 16
