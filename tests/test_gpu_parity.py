"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the
golden vectors produced by the reference itself.

Tolerances (fp32 path): single network call rel-RMS <= 1e-4;
full enhance rel-RMS <= 1e-3 and SI-SDR >= 60 dB against the reference output
on the same noise (drawn from the same seeded CPU generator).
"""
import math

import numpy as np
import pytest
import torch

from conftest import golden_state_dict, load_golden, rel_rms, si_sdr
from open_universe_amd import _lib as L
from open_universe_amd import engine as E
from open_universe_amd.configs import get_config
from open_universe_amd.networks.universe import Universe, UniverseGAN
from oracle import ou_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _model(tag, name, nch):
    d = load_golden(tag)
    cfg = get_config(name, nch)
    cls = UniverseGAN if cfg["_target_"].endswith("UniverseGAN") else Universe
    m = cls(**{k: v for k, v in cfg.items() if k != "_target_"})
    m.load_state_dict(golden_state_dict(d), strict=False)
    return d, cfg, m.to(DEV).eval()


@pytest.fixture(scope="module")
def pp16():
    return _model("pp16", "pp16", None)


@pytest.fixture(scope="module")
def pp16_c4():
    return _model("pp16_c4", "pp16", 4)


def _t(a):
    return torch.from_numpy(np.asarray(a))


def _dev(a):
    return _t(a).to(DEV)


# ----------------------------------------------------------------- layers
def _run_conv(cw, x, out_shape, form="folded", **kw):
    xa = E.Act(x.to(DEV).contiguous())
    y = E.new_act(*out_shape, DEV)
    d = E.conv_desc(cw, xa, y, **kw)
    if form == "fir":   # the FIR-applied kernels (tile bit 17) instead of the folded weights
        assert cw.fir is not None
        d = E.fir_desc(d)
    L.run_now(L.OP_CONV, d, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return y.t.cpu()


@pytest.mark.parametrize("lvl,T", [(0, 1000), (1, 517), (4, 33)])
@pytest.mark.parametrize("conv,k", [("conv1", 5), ("conv3", 3)])
def test_same_conv_layer(pp16, lvl, T, conv, k):
    d, cfg, m = pp16
    sd = {kk: v.cpu() for kk, v in m.state_dict().items()}
    p = f"_edm_model.encoder.ds_modules.{lvl}.{conv}"
    C = 32 * 2 ** min(lvl, 4)
    x = torch.randn(2, C, T, generator=torch.Generator().manual_seed(lvl))
    cw = E.prep_same(sd, p, k, DEV)
    y = _run_conv(cw, x, (2, C, T))
    ref = O.prelu_conv(sd, p, x, k, padding="same")
    assert rel_rms(y, ref) < 1e-5


@pytest.mark.parametrize("form", ["folded", "fir"])
@pytest.mark.parametrize("lvl,r", [(0, 2), (1, 4), (3, 5)])
def test_down_conv_layer(pp16, lvl, r, form):
    d, cfg, m = pp16
    sd = {kk: v.cpu() for kk, v in m.state_dict().items()}
    p = f"_edm_model.encoder.ds_modules.{lvl}.rate_change_conv"
    C = 32 * 2**lvl
    T = 203 * r + 1
    x = torch.randn(2, C, T, generator=torch.Generator().manual_seed(7))
    cw = E.prep_down(sd, p, r, True, DEV)
    U = -(-T // r)
    y = _run_conv(cw, x, (2, 2 * C, U), form=form)
    ref = O.prelu_conv(sd, p, x, r, stride=r, antialias=True)
    assert rel_rms(y, ref) < 1e-5


@pytest.mark.parametrize("form", ["folded", "fir"])
@pytest.mark.parametrize("lvl,r", [(1, 5), (2, 4), (4, 2)])
def test_up_conv_layer(pp16, lvl, r, form):
    d, cfg, m = pp16
    sd = {kk: v.cpu() for kk, v in m.state_dict().items()}
    p = f"_edm_model.decoder.up_modules.{lvl}.rate_change_conv"
    Cin = sd[p + ".conv.weight_v"].shape[0]
    Tin = 77
    x = torch.randn(1, Cin, Tin, generator=torch.Generator().manual_seed(3))
    res = torch.randn(1, Cin // 2, r * Tin, generator=torch.Generator().manual_seed(4))
    cw = E.prep_up(sd, p, r, True, DEV)
    resa = E.Act(res.to(DEV))
    y = _run_conv(cw, x, (1, Cin // 2, r * Tin), form=form, n_frames=Tin, valid_len=r * Tin, res1=resa,
                  s1=float(E.NF2))
    ref = (O.prelu_conv(sd, p, x, r, stride=r, transpose=True, antialias=True) + res) * E.NF2
    assert rel_rms(y, ref) < 1e-5


def test_gru_layer(pp16):
    d, cfg, m = pp16
    eng = m._get_engine()
    sd = {kk: v.cpu() for kk, v in m.state_dict().items()}
    T = 57
    x = torch.randn(2, 512, T, generator=torch.Generator().manual_seed(9)) * 0.5
    res = torch.randn(2, 512, T, generator=torch.Generator().manual_seed(10))
    xa, gi, y = E.Act(x.to(DEV)), E.new_act(2, 1536, T, DEV), E.new_act(2, 512, T, DEV)
    gran = torch.zeros(L.load().ou_gru_workspace_bytes(256, 2) // 8, dtype=torch.int64, device=DEV)
    prog = L.Program()
    E.rec_gru(prog, eng.s_gru, 0, xa, gi, y, gran, eng.status, res=E.Act(res.to(DEV)), res_scale=0.5)
    prog.run(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert int(eng.status.max()) == 0
    ref = (O.gru(sd, "_edm_model.encoder.gru", x, 1) + res) * 0.5
    assert rel_rms(y.t.cpu(), ref) < 1e-5


@pytest.mark.parametrize("Ts", [(2, 2, 2), (3, 3, 3), (4, 4, 4), (5, 5, 5), (6, 6, 6), (4, 6, 9), (3, 7, 2)])
def test_gru_ws_zeroed_short_launches_back_to_back(pp16, Ts):
    """Launches that skip the per-launch memset (ou_gru_desc.ws_zeroed) on one
    workspace zeroed once: a short launch's leftover step tags (T-1, T-2) must
    not satisfy the next launch's first polls (tags 1, 2) -- launches of fewer
    than 5 steps clear the workspace before and after they run, so launches
    of different T (4 then 6) share it too.  Each of three back-to-back
    launches must equal the same layer run alone with a per-launch memset."""
    d, cfg, m = pp16
    eng = m._get_engine()
    B = 2
    xs = [torch.randn(B, 512, T, generator=torch.Generator().manual_seed(20 + i)) * 0.5 for i, T in enumerate(Ts)]
    gran = torch.zeros(L.load().ou_gru_workspace_bytes(256, B) // 8, dtype=torch.int64, device=DEV)

    def run(ws_zeroed, inputs):
        saved, E._GRU_WS_ZEROED = E._GRU_WS_ZEROED, ws_zeroed
        try:
            prog = L.Program()
            if ws_zeroed:
                E.rec_gru_ws_zero(prog, gran)
            outs = []
            for x in inputs:
                T = x.shape[2]
                xa, gi, y = E.Act(x.to(DEV)), E.new_act(B, 1536, T, DEV), E.new_act(B, 512, T, DEV)
                E.rec_gru(prog, eng.s_gru, 0, xa, gi, y, gran, eng.status)
                outs.append((xa, gi, y))
            prog.run(torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
        finally:
            E._GRU_WS_ZEROED = saved
        assert int(eng.status.max()) == 0
        return [y.t.cpu() for _, _, y in outs]

    chained = run(True, xs)
    for x, yc in zip(xs, chained):
        alone = run(False, [x])[0]
        assert torch.equal(yc, alone)


@pytest.mark.parametrize("B,xcd", [(1, 2), (1, 7), (5, 3)])
def test_gru_xcd_offset_same_result(pp16, B, xcd):
    """ou_gru_desc.flags bits 12-14 (engine.rec_gru xcd=): the chains' XCD
    layout rotated by an offset (bit 15 keeps the default bits 0-11) computes
    the same recurrence bit for bit; B = 5 puts chains in two rows of 8."""
    d, cfg, m = pp16
    eng = m._get_engine()
    T = 97
    x = torch.randn(B, 512, T, generator=torch.Generator().manual_seed(31)) * 0.5
    gran = torch.zeros(L.load().ou_gru_workspace_bytes(256, B) // 8, dtype=torch.int64, device=DEV)

    def run(off):
        prog = L.Program()
        xa, gi, y = E.Act(x.to(DEV)), E.new_act(B, 1536, T, DEV), E.new_act(B, 512, T, DEV)
        E.rec_gru(prog, eng.s_gru, 0, xa, gi, y, gran, eng.status, xcd=off)
        prog.run(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert int(eng.status.max()) == 0
        return y.t.cpu()

    assert torch.equal(run(xcd), run(0))


# ----------------------------------------------------------------- networks
@pytest.mark.parametrize("tag,name,nch", [("pp16", "pp16", None), ("pp16_c4", "pp16", 4),
                                          ("orig16_c4", "orig16", 4), ("pp24_c4", "pp24", 4)])
def test_conditioner_vs_reference(tag, name, nch):
    d, cfg, m = _model(tag, name, nch)
    with torch.no_grad():
        conds, y_hat, h = m.condition_model(_dev(d["cond_in"]), train=True)
    for i, c in enumerate(conds):
        assert rel_rms(c.cpu(), d[f"cond_out{i}"]) < 1e-4, i
    assert rel_rms(y_hat.cpu(), d["cond_yhat"]) < 1e-4
    assert rel_rms(h.cpu(), d["cond_h"]) < 1e-4


@pytest.mark.parametrize("tag,name,nch", [("pp16", "pp16", None), ("pp16_c4", "pp16", 4),
                                          ("orig16_c4", "orig16", 4), ("pp24_c4", "pp24", 4)])
def test_score_network_vs_reference(tag, name, nch):
    d, cfg, m = _model(tag, name, nch)
    conds = [_dev(d[f"cond_out{i}"]) for i in range(5)]
    with torch.no_grad():
        out = m.get_score_model()(_dev(d["score_x"]), _dev(d["score_sigma"]), conds)
    assert rel_rms(out.cpu(), d["score_out"]) < 1e-4


# ----------------------------------------------------------------- sampler
@pytest.mark.parametrize("tag,name,nch", [("pp16", "pp16", None), ("pp16_c4", "pp16", 4),
                                          ("orig16_c4", "orig16", 4), ("pp24_c4", "pp24", 4)])
def test_enhance_vs_reference(tag, name, nch):
    d, cfg, m = _model(tag, name, nch)
    mix = _dev(d["enh_mix"])
    with torch.no_grad():
        out = m.enhance(mix[:, 0], rng=torch.Generator().manual_seed(1028282)).cpu()
        assert out.shape == d["enh_out"].shape
        assert rel_rms(out, d["enh_out"]) < 1e-3
        assert si_sdr(out, d["enh_out"]) > 60
        out2 = m.enhance(mix, n_steps=3, rng=torch.Generator().manual_seed(7), keep_rms=True).cpu()
        assert rel_rms(out2, d["enh2_out"]) < 1e-3
        out3 = m.enhance(mix, target=_dev(d["enh_tgt"]), fake_score_snr=20.0,
                         rng=torch.Generator().manual_seed(11)).cpu()
        assert rel_rms(out3, d["enh_fake_out"]) < 1e-4


def test_enhance_options_vs_reference(pp16_c4):
    d, cfg, m = pp16_c4
    mix = _dev(d["enh_mix"])
    with torch.no_grad():
        ens = m.enhance(mix[0, 0], rng=torch.Generator().manual_seed(3), ensemble=3,
                        ensemble_stat="median").cpu()
        assert ens.shape == d["enh_ens_out"].shape
        assert rel_rms(ens, d["enh_ens_out"]) < 1e-3
        aux = m.enhance(mix, rng=torch.Generator().manual_seed(4), use_aux_signal=True).cpu()
        assert rel_rms(aux, d["enh_aux_out"]) < 1e-4
        warm = m.enhance(mix, rng=torch.Generator().manual_seed(6), warm_start=4).cpu()
        assert rel_rms(warm, d["enh_warm_out"]) < 1e-3


def test_graph_replay_equals_eager_and_is_deterministic(pp16_c4):
    d, cfg, m = pp16_c4
    mix = _dev(d["enh_mix"])
    from open_universe_amd.plan import EnhancePlan

    eng = m._get_engine()
    plan = EnhancePlan(eng, 2, mix.shape[-1], 8, 1.3)
    a = plan(mix, torch.Generator(device=DEV).manual_seed(5), use_graph=False).clone()
    b = plan(mix, torch.Generator(device=DEV).manual_seed(5), use_graph=True).clone()
    c = plan(mix, torch.Generator(device=DEV).manual_seed(5), use_graph=True).clone()
    assert torch.equal(a, b) and torch.equal(b, c)


def test_enhance_full_size_properties(pp16):
    """BASELINE config C2 shape (8 s at 16 kHz, B = 2): size-independent
    properties -- finite, bounded by the peak normaliser, deterministic, and
    batch items independent of each other.  (The value comparison against the
    oracle at this size is test_gpu_parity_sizes.test_c2_size_enhance_vs_oracle.)"""
    d, cfg, m = pp16
    T = 128000
    g = torch.Generator().manual_seed(0)
    mix = (0.1 * torch.randn(2, T, generator=g)).to(DEV)
    with torch.no_grad():
        a = m.enhance(mix, rng=torch.Generator(device=DEV).manual_seed(1))
        b = m.enhance(mix, rng=torch.Generator(device=DEV).manual_seed(1))
        assert torch.isfinite(a).all() and a.abs().max() <= 1.0
        assert torch.equal(a, b)
        # item 1 alone, with the noise item 1 saw inside the batch
        plan = next(p for k, p in m._plans.items() if k[0] == 2 and k[1] == T)
        nz = plan.NZ[:, 1:2].clone()
        from open_universe_amd.plan import EnhancePlan

        p1 = EnhancePlan(m._get_engine(), 1, T, 8, 1.3)
        p1.MIX.copy_(mix[1:2, None])
        p1.NZ.copy_(nz)
        p1._launch(torch.cuda.current_stream().cuda_stream, True)
        torch.cuda.synchronize()
        # different batch sizes may autotune to different tiles (summation order)
        assert rel_rms(p1.OUT[0].cpu(), a[1].cpu()) < 1e-4


# ------------------------------------------------------- operand precision
def test_enhance_f32_operands_vs_reference(monkeypatch):
    """The f32-operand ou_conv build (OUHIP_CONV_PREC=f32) against the
    reference at the same bar as the default split-f16 build above."""
    monkeypatch.setenv("OUHIP_CONV_PREC", "f32")
    d, cfg, m = _model("pp16", "pp16", None)
    assert m._get_engine().conv_prec == 0
    mix = _dev(d["enh_mix"])
    with torch.no_grad():
        out = m.enhance(mix[:, 0], rng=torch.Generator().manual_seed(1028282)).cpu()
    assert rel_rms(out, d["enh_out"]) < 1e-3
    assert si_sdr(out, d["enh_out"]) > 60


def test_split_and_f32_operands_agree_full_size(pp16, monkeypatch):
    """BASELINE C2 size (8 s, 16 kHz, B = 1): the split-f16 and the f32 operand
    builds of the whole enhance() agree to f32 summation-order level."""
    d, cfg, m = pp16
    assert m._get_engine().conv_prec == 1
    T = 128000
    mix = (0.1 * torch.randn(1, T, generator=torch.Generator().manual_seed(3))).to(DEV)
    monkeypatch.setenv("OUHIP_CONV_PREC", "f32")
    d32, _, m32 = _model("pp16", "pp16", None)
    with torch.no_grad():
        a = m.enhance(mix, rng=torch.Generator(device=DEV).manual_seed(2)).cpu()
        b = m32.enhance(mix, rng=torch.Generator(device=DEV).manual_seed(2)).cpu()
    assert torch.isfinite(a).all()
    assert rel_rms(a, b) < 1e-3 and si_sdr(a, b) > 60


@pytest.mark.parametrize("shift", [4, 13])
def test_enhance_widened_exponents_vs_reference(shift):
    """Every split-f16 operand staged at a non-default exponent (ConvDesc
    xs_shift / sy_shift, ou_block_desc.shift -- what Engine.widen_ranges
    moves a flagged layer to): the result scaling 2^(s - 6) is right in every
    kernel family, and the enhance still matches the reference."""
    d, cfg, m = _model("pp16_c4", "pp16", 4)
    eng = m._get_engine()
    for o in eng.range_owners:
        if hasattr(o, "xshift"):
            o.xshift = shift
        else:
            o.shifts = [shift] * 4
    mix = _dev(d["enh_mix"])
    with torch.no_grad():
        out = m.enhance(mix[:, 0], rng=torch.Generator().manual_seed(1028282)).cpu()
    assert eng.conv_prec == 1 and m.range_fallbacks == 0 and m.range_widenings == 0
    assert rel_rms(out, d["enh_out"]) < 1e-3
    assert si_sdr(out, d["enh_out"]) > 60


def test_enhance_f16_operands_vs_reference(monkeypatch):
    """OUHIP_CONV_PREC=f16 (BASELINE configs[4]): f16 conv operands with f32
    accumulation, against the f32 reference: SI-SDR >= 30 dB."""
    monkeypatch.setenv("OUHIP_CONV_PREC", "f16")
    d, cfg, m = _model("pp16", "pp16", None)
    assert m._get_engine().conv_prec == 2
    mix = _dev(d["enh_mix"])
    with torch.no_grad():
        out = m.enhance(mix[:, 0], rng=torch.Generator().manual_seed(1028282)).cpu()
    # no range-flag rerun in f32: the f16 path itself produced this output
    assert m._get_engine().conv_prec == 2
    assert int(m._get_engine().status.abs().sum()) == 0
    assert torch.isfinite(out).all()
    assert si_sdr(out, d["enh_out"]) > 30
