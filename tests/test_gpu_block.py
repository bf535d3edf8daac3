"""ou_block (fused ConvBlock main path) against the unfused ou_conv sequence
and a float64 torch evaluation of the reference arithmetic
(blocks.py:393-416): every supported channel count, every optional epilogue
input, lengths that are not multiples of the workgroup's frame count (and
shorter than it), batch 2, f32, split-f16 and f16 operands."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from open_universe_amd import _lib as L
from open_universe_amd import engine as E

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _specs(C, g):
    out = []
    for k in (5, 3, 3):
        w = torch.randn(C, C, k, generator=g) / np.sqrt(C * k)
        b = 0.1 * torch.randn(C, generator=g)
        slope = float(0.05 + 0.4 * torch.rand(1, generator=g))
        out.append(E.ConvSpec(w.numpy(), C, 1, (k - 1) // 2, 1, slope, b.numpy(), ref_macs=float(w.numel())))
    return out


def _ref(specs, h, sc=None, film=None, res2=None, s2=1.0):
    """float64 restatement: PReLU -> conv (zero 'same' padding) -> bias."""
    def pc(sp, x):
        x = torch.where(x >= 0, x, sp.slope * x)
        w = torch.from_numpy(sp.w).double()
        return F.conv1d(x, w, padding=sp.pad) + torch.from_numpy(sp.bias).double()[None, :, None]

    r = 0.5 ** 0.5
    c1 = pc(specs[0], h)
    if sc is not None:
        c1 = (c1 + sc) * r
    if film is not None:
        C = h.shape[1]
        c1 = film[:, :C, None] * c1 + film[:, C:, None]
    y = (h + pc(specs[2], pc(specs[1], c1))) * r
    if res2 is not None:
        y = (y + res2) * s2
    return y, c1


def _run(bw, h, out, fused, **kw):
    keep = bw.fused
    if not fused:
        bw.fused = None
    try:
        prog = L.Program()
        tA = E.new_act(h.B, h.C, h.T, DEV)
        tB = E.new_act(h.B, h.C, h.T, DEV)
        E.rec_block(prog, bw, h, out, tA, tB, **kw)
        kinds = prog.op_kinds()
        prog.run(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    finally:
        bw.fused = keep
    return kinds


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm())


@pytest.mark.parametrize("prec", [0, 1, 2])
@pytest.mark.parametrize("C,T", [(32, 1000), (32, 7), (64, 300), (64, 60), (128, 125), (128, 29), (128, 3),
                                 (48, 700), (48, 5), (96, 500), (96, 9), (192, 241), (192, 61)])
@pytest.mark.parametrize("mode", ["plain", "score_dec", "cond_dec", "res2"])
def test_block_vs_unfused_and_reference(C, T, mode, prec):
    g = torch.Generator().manual_seed(C * 1000 + T)
    specs = _specs(C, g)
    B = 2
    status = torch.zeros(4, dtype=torch.int32, device=DEV)
    saved = E._PREP_STATUS
    E._PREP_STATUS = status.data_ptr() + 4
    try:
        cws = [E.make_conv(sp, DEV, prec=prec) for sp in specs]
        fused = E.prep_fused(specs, C, prec, DEV)
    finally:
        E._PREP_STATUS = saved
    assert fused is not None
    bw = E.BlockW(C, "none", None, *cws, None, fused)
    h = torch.randn(B, C, T, generator=g)
    sc = torch.randn(B, C, T, generator=g) if mode == "score_dec" else None
    film = (1.0 + 0.3 * torch.randn(B, 2 * C, generator=g)) if mode == "score_dec" else None
    res2 = torch.randn(B, C, T, generator=g) if mode == "res2" else None
    ref, c1 = _ref(specs, h.double(), None if sc is None else sc.double(),
                   None if film is None else film.double(), None if res2 is None else res2.double(), 0.7)
    ha = E.Act(h.to(DEV))
    kw = {}
    film_dev = film.to(DEV) if film is not None else None   # referenced until the launches ran
    if sc is not None:
        kw.update(sc=E.Act(sc.to(DEV)), film=film_dev.data_ptr(), film_bs=2 * C)
    if res2 is not None:
        kw.update(res2=E.Act(res2.to(DEV)), s2=0.7)
    outs = {}
    for fz in (True, False):
        out = E.new_act(B, C, T, DEV)
        co = E.new_act(B, C, T, DEV) if mode == "cond_dec" else None
        kinds = _run(bw, ha, out, fz, cond_out=co, **kw)
        assert (L.OP_BLOCK in kinds) == fz
        outs[fz] = (out.t.clone(), None if co is None else co.t.clone())
    assert int(status.abs().sum()) == 0
    tol = 1e-5 if prec in (0, 1) else 3e-3   # f32 and split-f16 operands: f32-class; f16: 11 bits
    assert _rel(outs[True][0], ref) < tol
    assert _rel(outs[True][0], outs[False][0]) < tol
    if mode == "cond_dec":
        assert _rel(outs[True][1], c1) < tol


def test_block_range_flag():
    """A staged input beyond the split-f16 range sets the status word."""
    C, T = 64, 200
    g = torch.Generator().manual_seed(1)
    specs = _specs(C, g)
    status = torch.zeros(4, dtype=torch.int32, device=DEV)
    saved = E._PREP_STATUS
    E._PREP_STATUS = status.data_ptr() + 4
    try:
        cws = [E.make_conv(sp, DEV, prec=1) for sp in specs]
    finally:
        E._PREP_STATUS = saved
    bw = E.BlockW(C, "none", None, *cws, None, E.prep_fused(specs, C, 1, DEV))
    h = torch.randn(1, C, T, generator=g)
    h[0, 3, 50] = 3.0e6
    out = E.new_act(1, C, T, DEV)
    _run(bw, E.Act(h.to(DEV)), out, True)
    assert int(status[1]) == 1


@pytest.mark.parametrize("name", ["pp16", "pp24"])
def test_score_ends_fused_equal_unfused(monkeypatch, name):
    """The score input conv fused into the first encoder block and the head
    (EDM wrapper + sampler update) fused into the last decoder block give the
    same enhance as separate ou_conv / ou_head launches (f32 summation-order
    level), and the fused program has fewer launches.  PP24's level-0 blocks
    have 48 channels: padded MFMA rows in the fused input conv and head."""
    from conftest import golden_state_dict, load_golden
    from open_universe_amd.configs import get_config
    from open_universe_amd.networks.universe import UniverseGAN

    d = load_golden(name)
    outs, nops = {}, {}
    for fuse in ("1", "0"):
        monkeypatch.setenv("OUHIP_FUSE_ENDS", fuse)
        cfg = get_config(name, None)
        m = UniverseGAN(**{k: v for k, v in cfg.items() if k != "_target_"})
        m.load_state_dict(golden_state_dict(d), strict=False)
        m = m.to(DEV).eval()
        mix = torch.from_numpy(d["enh_mix"]).to(DEV)
        with torch.no_grad():
            outs[fuse] = m.enhance(mix[:, 0], rng=torch.Generator().manual_seed(1028282)).cpu()
            sc = m.get_score_model()(torch.from_numpy(d["score_x"]).to(DEV), torch.from_numpy(d["score_sigma"]).to(DEV),
                                     [torch.from_numpy(d[f"cond_out{i}"]).to(DEV) for i in range(5)]).cpu()
        nops[fuse] = len(next(iter(m._plans.values())).prog)
        assert _rel(sc, torch.from_numpy(d["score_out"])) < 1e-4
    assert _rel(outs["1"], outs["0"]) < 1e-5
    assert nops["1"] < nops["0"]


def _down_spec(C, r, kt, g):
    """A strided rate-change conv in the engine's frame-view form (spec_down):
    w[2C][ci*r + ph][kt], zero padding; kt 3 is centred (frames -1, 0, +1)."""
    w = torch.randn(2 * C, C * r, kt, generator=g) / np.sqrt(C * r * kt)
    b = 0.1 * torch.randn(2 * C, generator=g)
    return E.ConvSpec(w.numpy(), C, r, (kt - 1) // 2, 1, 0.2, b.numpy(), ref_macs=float(w.numel()))


def _down_ref(sp, y):
    """float64: PReLU, zero right-pad to a multiple of r, frame view, conv."""
    r, kt = sp.frame, sp.w.shape[2]
    B, C, T = y.shape
    U = -(-T // r)
    x = torch.where(y >= 0, y, sp.slope * y)
    x = F.pad(x, (0, U * r - T)).reshape(B, C, U, r).permute(0, 1, 3, 2).reshape(B, C * r, U)
    w = torch.from_numpy(sp.w).double()
    return F.conv1d(x, w, padding=(kt - 1) // 2) + torch.from_numpy(sp.bias).double()[None, :, None]


@pytest.mark.parametrize("prec", [1, 2])
@pytest.mark.parametrize("C,r,kt,T", [(32, 2, 3, 1001), (32, 2, 3, 119), (32, 2, 3, 3), (32, 2, 1, 250),
                                      (64, 4, 1, 503), (64, 4, 1, 61), (64, 4, 1, 5)])
def test_block_fused_down(C, r, kt, T, prec):
    """The encoder's rate-change conv as ou_block's fourth stage: the block
    output y and e = rate_conv(y) against the unfused launches and float64,
    ragged lengths (the last workgroup's frames, a partial last output
    frame), batch 2, with and without FiLM."""
    g = torch.Generator().manual_seed(C + r + kt + T)
    specs = _specs(C, g)
    rsp = _down_spec(C, r, kt, g)
    cws = [E.make_conv(sp, DEV, prec=prec) for sp in specs]
    rc = E.make_conv(rsp, DEV, prec=prec)
    fused = E.prep_fused(specs, C, prec, DEV)
    down = E.prep_down_fused(rsp, C, prec, rc.bias, DEV)
    assert fused is not None and down is not None
    bw = E.BlockW(C, "down", r, *cws, rc, fused, down)
    B = 2
    h = torch.randn(B, C, T, generator=g)
    film = torch.randn(B, 2 * C, generator=g) * 0.5 + torch.cat([torch.ones(C), torch.zeros(C)])
    U = -(-T // r)
    filmd = film.to(DEV)
    for use_film in (False, True):
        kw = {"film": filmd.data_ptr(), "film_bs": 2 * C} if use_film else {}
        res = {}
        for fz in ("fused", "unfused"):
            if fz == "unfused":
                bw.down = None
            out, e = E.new_act(B, C, T, DEV), E.new_act(B, 2 * C, U, DEV)
            kinds = _run(bw, E.Act(h.to(DEV)), out, True, e_out=e, **kw)
            bw.down = down
            res[fz] = (out.t.cpu(), e.t.cpu(), kinds)
        assert res["fused"][2].count(L.OP_CONV) == 0 and res["unfused"][2].count(L.OP_CONV) == 1
        y_ref, _ = _ref(specs, h.double(), film=film.double() if use_film else None)
        e_ref = _down_ref(rsp, y_ref)
        tol = 1e-5 if prec == 1 else 3e-3
        assert _rel(res["fused"][0], y_ref) < tol
        assert _rel(res["fused"][1], e_ref) < tol, _rel(res["fused"][1], e_ref)
        assert _rel(res["fused"][1], res["unfused"][1]) < tol


def test_encoder_down_fused_equal_unfused(monkeypatch):
    """The encoders' rate-change convs fused into their blocks (score and
    conditioner, 32 and 64 channels) give the same enhance as separate
    launches, the score network still matches the reference's output, and the
    fused program has fewer launches."""
    from conftest import golden_state_dict, load_golden
    from open_universe_amd.configs import get_config
    from open_universe_amd.networks.universe import UniverseGAN

    d = load_golden("pp16")
    outs, nops = {}, {}
    for fuse in ("1", "0"):
        monkeypatch.setenv("OUHIP_FUSE_DOWN", fuse)
        cfg = get_config("pp16", None)
        m = UniverseGAN(**{k: v for k, v in cfg.items() if k != "_target_"})
        m.load_state_dict(golden_state_dict(d), strict=False)
        m = m.to(DEV).eval()
        mix = torch.from_numpy(d["enh_mix"]).to(DEV)
        with torch.no_grad():
            outs[fuse] = m.enhance(mix[:, 0], rng=torch.Generator().manual_seed(1028282)).cpu()
            sc = m.get_score_model()(torch.from_numpy(d["score_x"]).to(DEV), torch.from_numpy(d["score_sigma"]).to(DEV),
                                     [torch.from_numpy(d[f"cond_out{i}"]).to(DEV) for i in range(5)]).cpu()
        nops[fuse] = len(next(iter(m._plans.values())).prog)
        assert _rel(sc, torch.from_numpy(d["score_out"])) < 1e-4
    assert _rel(outs["1"], outs["0"]) < 1e-5
    assert nops["1"] <= nops["0"] - 3
