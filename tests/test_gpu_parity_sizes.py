"""GPU parity at the real sizes: full-width ORIG16 / PP24 against the
reference's own fixtures, GRU layers at every hidden size / batch the configs
run against torch.nn.GRU fixtures, the ensemble reductions against the
reference, and the HIP enhance against the pinned CPU oracle at the BASELINE
configs' shapes (C2 8 s, C3 60 steps B=8, C4 PP24 full width, C5 60 s f16)
with the same injected noise (one seeded CPU generator, drawn in the
reference's order on both sides).

Tolerances: fp32 enhance rel-RMS <= 1e-3 and SI-SDR >= 60 dB
against the reference / oracle; per network call rel-RMS <= 1e-4; GRU layer
rel-RMS <= 1e-5; the fp16 config SI-SDR >= 30 dB against the fp32 oracle.
"""
import numpy as np
import pytest
import torch

from conftest import golden_state_dict, load_golden, rel_rms, si_sdr
from open_universe_amd import _lib as L
from open_universe_amd import engine as E
from open_universe_amd.configs import get_config
from open_universe_amd.networks.universe import Universe, UniverseGAN
from open_universe_amd.utils.synthetic import synth_audio, synth_state_dict, synth_tensor
from oracle import ou_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
torch.set_num_threads(16)   # the oracle legs: the GPU box's host share


def _t(a):
    return torch.from_numpy(np.asarray(a))


def _golden_model(tag, name, nch=None):
    d = load_golden(tag)
    cfg = get_config(name, nch)
    cls = UniverseGAN if cfg["_target_"].endswith("UniverseGAN") else Universe
    m = cls(**{k: v for k, v in cfg.items() if k != "_target_"})
    m.load_state_dict(golden_state_dict(d), strict=False)
    return d, cfg, m.to(DEV).eval()


def _synth_model(name, seed=0):
    cfg = get_config(name, None)
    cls = UniverseGAN if cfg["_target_"].endswith("UniverseGAN") else Universe
    m = cls(**{k: v for k, v in cfg.items() if k != "_target_"})
    m.load_state_dict(synth_state_dict([(k, v.shape) for k, v in m.state_dict().items()], seed), strict=False)
    return cfg, m.to(DEV).eval()


def _oracle(m, cfg):
    return O.Oracle({k: v.detach().cpu() for k, v in m.state_dict().items()}, cfg)


def _clips(B, seconds, fs, base=0):
    T = int(seconds * fs)
    return torch.from_numpy(np.stack([synth_audio(T, fs, base + j)[0] for j in range(B)]))


# ----------------------------------------------------------------- GRU layers
@pytest.mark.parametrize("case", ["h384_b8", "h384_b32", "h128_b32", "h64_b8_l2"])
def test_gru_layers_vs_torch_gru(case):
    """ou_gru (with its ou_conv input projection) against torch.nn.GRU at
    H = 384 (PP24, C4 batch 32), 128 and 64 (two layers, as the conditioner)."""
    d = load_golden("gru")
    H, layers, B, T = (int(v) for v in d[f"{case}_meta"])
    p = f"gru_{case}"
    sd = {}
    for l in range(layers):
        for sfx in ("", "_reverse"):
            for kind, shape in (("weight_ih", (3 * H, 2 * H)), ("weight_hh", (3 * H, H)),
                                ("bias_ih", (3 * H,)), ("bias_hh", (3 * H,))):
                n = f"{p}.{kind}_l{l}{sfx}"
                sd[n] = synth_tensor(n, shape)
    for prec in (0, 1):   # f32 and split-f16 input projection
        saved, E._PREP_PREC = E._PREP_PREC, prec
        try:
            gw = E.prep_gru(sd, p, layers, DEV)
        finally:
            E._PREP_PREC = saved
        status = torch.zeros(4, dtype=torch.int32, device=DEV)
        gran = torch.zeros(L.load().ou_gru_workspace_bytes(H, B) // 8, dtype=torch.int64, device=DEV)
        x = E.Act(_t(d[f"{case}_x"]).to(DEV).contiguous())
        gi = E.new_act(B, 6 * H, T, DEV)
        prog = L.Program()
        h = x
        for l in range(layers):
            y = E.new_act(B, 2 * H, T, DEV)
            E.rec_gru(prog, gw, l, h, gi, y, gran, status)
            h = y
        prog.run(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert int(status.abs().sum()) == 0
        assert rel_rms(h.t.cpu(), d[f"{case}_y"]) < 1e-5, prec


# ----------------------------------------------------------------- ensembles
@pytest.mark.parametrize("E_", [1, 2, 3, 4, 5, 8, 16, 17, 32])
def test_signal_median_kernel_vs_oracle(E_):
    """Bit-exact against the restated reference.  Batch item 1 has many exact
    ties between members: the kernel ranks ties by member index (a stable
    sort), which is what torch's CPU sort does for up to 16 members; beyond
    that torch's sort is unstable, so item 1 is compared only for E <= 16."""
    g = torch.Generator().manual_seed(E_)
    x = torch.randn(E_, 3, 1, 5003, generator=g)
    x[:, 1] = torch.round(x[:, 1] * 2) / 2   # many ties across members
    from open_universe_amd.utils.stats import ensemble_reduce, signal_median

    got = signal_median(x.to(DEV)).cpu()
    want = O.signal_median(x)
    items = [0, 1, 2] if E_ <= 16 else [0, 2]
    assert torch.equal(got[items], want[items])
    assert torch.allclose(ensemble_reduce(x.to(DEV), "mean").cpu(), x.mean(0), rtol=1e-6, atol=1e-7)
    assert torch.equal(ensemble_reduce(x.to(DEV), "median").cpu(), x.median(0).values)


def test_ensemble_mean_and_signal_median_vs_reference():
    d, cfg, m = _golden_model("pp16_c4", "pp16", 4)
    mix = _t(d["enh_mix"]).to(DEV)
    with torch.no_grad():
        mean = m.enhance(mix[0, 0], rng=torch.Generator().manual_seed(3), ensemble=3,
                         ensemble_stat="mean").cpu()
        assert mean.shape == d["enh_ensmean_out"].shape
        assert rel_rms(mean, d["enh_ensmean_out"]) < 1e-3
        for e, seed in ((3, 8), (4, 9)):
            sm = m.enhance(mix, rng=torch.Generator().manual_seed(seed), ensemble=e,
                           ensemble_stat="signal_median").cpu()
            assert sm.shape == d[f"enh_sigmed{e}_out"].shape
            assert rel_rms(sm, d[f"enh_sigmed{e}_out"]) < 1e-3
        # the known-answer mode reduces through the same kernels (one item: the
        # reference broadcasts target against the repeated mixture)
        fk = m.enhance(mix[:1], target=_t(d["enh_tgt"])[:1].to(DEV), fake_score_snr=20.0,
                       rng=torch.Generator().manual_seed(11), ensemble=3, ensemble_stat="signal_median")
        assert fk.shape == mix[:1].shape and torch.isfinite(fk).all()


# ------------------------------------------------------- full-width fixtures
@pytest.mark.parametrize("tag,name", [("orig16", "orig16"), ("pp24", "pp24")])
def test_full_width_networks_vs_reference(tag, name):
    d, cfg, m = _golden_model(tag, name)
    with torch.no_grad():
        conds, y_hat, h = m.condition_model(_t(d["cond_in"]).to(DEV), train=True)
        for i, c in enumerate(conds):
            assert rel_rms(c.cpu(), d[f"cond_out{i}"]) < 1e-4, i
        conds = [_t(d[f"cond_out{i}"]).to(DEV) for i in range(5)]
        out = m.get_score_model()(_t(d["score_x"]).to(DEV), _t(d["score_sigma"]).to(DEV), conds)
    assert rel_rms(out.cpu(), d["score_out"]) < 1e-4


def test_full_width_orig16_enhance_8_and_60_steps():
    """ORIG16 (BASELINE configs[2]'s model) at full width: the default sampler
    and the 60-step sampler against the reference."""
    d, cfg, m = _golden_model("orig16", "orig16")
    mix = _t(d["enh_mix"]).to(DEV)
    with torch.no_grad():
        out = m.enhance(mix[:, 0], rng=torch.Generator().manual_seed(1028282)).cpu()
        assert rel_rms(out, d["enh_out"]) < 1e-3 and si_sdr(out, d["enh_out"]) > 60
        out60 = m.enhance(mix[:, 0], n_steps=60, rng=torch.Generator().manual_seed(60)).cpu()
    assert rel_rms(out60, d["enh60_out"]) < 1e-3 and si_sdr(out60, d["enh60_out"]) > 60
    assert m._get_engine().conv_prec == 1


def test_full_width_pp24_enhance():
    """PP24 at full width (48..768 channels, GRU H = 384).  With the seeded
    synthetic weights the reference's activations reach ~8e6 (fixture
    enh_peak_activation), beyond the split-f16 range at the default 2^-6
    staging exponent: the range flags name the layers, the engine widens only
    their exponents and reruns the same enhance on split-f16 operands (no f32
    fallback), which must match the reference."""
    d, cfg, m = _golden_model("pp24", "pp24")
    assert float(d["enh_peak_activation"]) > 2.0**21
    mix = _t(d["enh_mix"]).to(DEV)
    with torch.no_grad():
        out = m.enhance(mix[:, 0], rng=torch.Generator().manual_seed(1028282)).cpu()
    eng = m._get_engine()
    assert eng.conv_prec == 1 and m.range_fallbacks == 0   # still split-f16
    # reported (bench.py "widenings").  One replay names only the first
    # layers to overflow: their inf / NaN hides the layers behind them, which
    # the next rerun names (OUHIP_RANGE_LOG=1: 2 + 7 + 4 layers over 3 reruns)
    assert 1 <= m.range_widenings <= 3
    wide = [o for o in eng.range_owners if (getattr(o, "xshift", 6) != 6 or any(x != 6 for x in
                                                                                  getattr(o, "shifts", [6])))]
    assert 0 < len(wide) < len(eng.range_owners) // 2       # only the flagged layers moved
    assert rel_rms(out, d["enh_out"]) < 1e-3 and si_sdr(out, d["enh_out"]) > 60
    w0 = m.range_widenings
    with torch.no_grad():   # the widened exponents stay: no second rerun, same bits
        out2 = m.enhance(mix[:, 0], rng=torch.Generator().manual_seed(1028282)).cpu()
    assert m.range_widenings == w0 and m.range_fallbacks == 0 and torch.equal(out2, out)


def test_full_width_pp24_damped_split_f16_vs_reference():
    """PP24 at full width with the damped synthetic family (pp24d: the
    reference's activations stay below 2^15): the production split-f16
    operands on the 48..768-channel geometries at rates 3 and 8 -- no f32
    rerun -- against the reference's networks and enhance."""
    d, cfg, m = _golden_model("pp24d", "pp24")
    assert float(d["enh_peak_activation"]) < 2.0**15
    with torch.no_grad():
        conds, y_hat, h = m.condition_model(_t(d["cond_in"]).to(DEV), train=True)
        for i, c in enumerate(conds):
            assert rel_rms(c.cpu(), d[f"cond_out{i}"]) < 1e-4, i
        conds = [_t(d[f"cond_out{i}"]).to(DEV) for i in range(5)]
        sc = m.get_score_model()(_t(d["score_x"]).to(DEV), _t(d["score_sigma"]).to(DEV), conds)
        assert rel_rms(sc.cpu(), d["score_out"]) < 1e-4
        mix = _t(d["enh_mix"]).to(DEV)
        out = m.enhance(mix[:, 0], rng=torch.Generator().manual_seed(1028282)).cpu()
        assert m._get_engine().conv_prec == 1   # split-f16 ran it, no f32 rerun
        assert rel_rms(out, d["enh_out"]) < 1e-3 and si_sdr(out, d["enh_out"]) > 60
        out2 = m.enhance(mix, n_steps=3, rng=torch.Generator().manual_seed(7), keep_rms=True).cpu()
        assert rel_rms(out2, d["enh2_out"]) < 1e-3 and si_sdr(out2, d["enh2_out"]) > 60
    assert m._get_engine().conv_prec == 1


@pytest.mark.parametrize("tag,name", [("pp16", "pp16"), ("pp24d", "pp24")])
def test_full_width_aux_and_warm_start_vs_reference(tag, name):
    """use_aux_signal and warm_start at full width (T = 3,360 / 5,040): the
    ou_snake_aa kernel over the 32- / 48-channel decoder output upsampled 2x,
    then the 1-channel conv, and the warm-started sampler, against the
    reference (universe.py:317-331, universe_gan.py:147-151)."""
    d, cfg, m = _golden_model(tag, name)
    mix = _t(d["enh_mix"]).to(DEV)
    with torch.no_grad():
        aux = m.enhance(mix, rng=torch.Generator().manual_seed(4), use_aux_signal=True).cpu()
        assert aux.shape == d["enh_aux_out"].shape
        assert rel_rms(aux, d["enh_aux_out"]) < 1e-4
        warm = m.enhance(mix, rng=torch.Generator().manual_seed(6), warm_start=4).cpu()
        assert rel_rms(warm, d["enh_warm_out"]) < 1e-3 and si_sdr(warm, d["enh_warm_out"]) > 60
    assert m._get_engine().conv_prec == 1


def test_c4_real_shape_damped_split_f16_item0_vs_oracle():
    """BASELINE configs[3] at its real shape: PP24 full width, batch 32, 10 s
    clips, damped synthetic weights, split-f16 operands.  The whole batch runs
    on the GPU; item 0 is compared with the fp32 oracle on the same noise
    slice (the oracle at B = 32 x 10 s would take minutes)."""
    from open_universe_amd.utils.synthetic import RC_DAMP

    cfg = get_config("pp24", None)
    m = UniverseGAN(**{k: v for k, v in cfg.items() if k != "_target_"})
    m.load_state_dict(synth_state_dict([(k, v.shape) for k, v in m.state_dict().items()], 0, RC_DAMP),
                      strict=False)
    m = m.to(DEV).eval()
    mix = _clips(32, 10.0, cfg["fs"], base=31)
    with torch.no_grad():
        out = m.enhance(mix.to(DEV), rng=torch.Generator().manual_seed(2024)).cpu()
        eng = m._get_engine()
        assert eng.conv_prec == 1 and int(eng.status.abs().sum()) == 0
        assert out.shape == (32, 240000) and torch.isfinite(out).all()
        nz = next(iter(m._plans.values())).NZ.cpu()   # (draws, 32, 1, Tp): the noise the GPU used
        it = iter(range(nz.shape[0]))
        ref = _oracle(m, cfg).enhance(mix[:1], noise_fn=lambda shp: nz[next(it), :1].reshape(shp))
    assert rel_rms(out[:1], ref) < 1e-3 and si_sdr(out[:1], ref) > 60
    # the other items are not copies of item 0
    assert rel_rms(out[1:2], out[:1]) > 0.1


def test_c4_real_shape_undamped_split_f16_item0_vs_oracle():
    """BASELINE configs[3] at its real shape on the UNDAMPED synthetic PP24
    weights (the bench's --undamped line): batch 32, 10 s clips.  The range
    flags widen the staging exponents of the layers that overflow (at most
    three reruns of the same noise), the batch stays on split-f16 operands,
    and item 0 matches the fp32 oracle on the same noise slice."""
    cfg, m = _synth_model("pp24", 0)
    mix = _clips(32, 10.0, cfg["fs"], base=31)
    with torch.no_grad():
        out = m.enhance(mix.to(DEV), rng=torch.Generator().manual_seed(2024)).cpu()
        eng = m._get_engine()
        assert eng.conv_prec == 1 and m.range_fallbacks == 0 and m.range_widenings <= 3
        assert int(eng.status.abs().sum()) == 0
        assert out.shape == (32, 240000) and torch.isfinite(out).all()
        nz = next(iter(m._plans.values())).NZ.cpu()   # (draws, 32, 1, Tp): the noise the GPU used
        it = iter(range(nz.shape[0]))
        ref = _oracle(m, cfg).enhance(mix[:1], noise_fn=lambda shp: nz[next(it), :1].reshape(shp))
    assert rel_rms(out[:1], ref) < 1e-3 and si_sdr(out[:1], ref) > 60
    assert rel_rms(out[1:2], out[:1]) > 0.1


def test_c3_real_shape_item0_vs_oracle():
    """BASELINE configs[2] at its benched geometry: ORIG16 full width, batch 8,
    8 s clips, 60 diffusion steps (universe.py:301-343 with n_steps=60), split-
    f16 operands, the whole batch on the GPU; item 0 against the fp32 oracle on
    the same noise slice (about 10 s of host time)."""
    cfg, m = _synth_model("orig16", 0)
    mix = _clips(8, 8.0, cfg["fs"], base=41)
    with torch.no_grad():
        out = m.enhance(mix.to(DEV), n_steps=60, rng=torch.Generator().manual_seed(2026)).cpu()
        eng = m._get_engine()
        assert eng.conv_prec == 1 and int(eng.status.abs().sum()) == 0 and m.range_fallbacks == 0
        assert out.shape == (8, 128000) and torch.isfinite(out).all()
        nz = next(iter(m._plans.values())).NZ.cpu()   # (draws, 8, 1, Tp): the noise the GPU used
        it = iter(range(nz.shape[0]))
        ref = _oracle(m, cfg).enhance(mix[:1], n_steps=60, noise_fn=lambda shp: nz[next(it), :1].reshape(shp))
    assert rel_rms(out[:1], ref) < 1e-3 and si_sdr(out[:1], ref) > 60
    assert rel_rms(out[1:2], out[:1]) > 0.1


# ------------------------------------------- BASELINE shapes vs the oracle
def _vs_oracle(name, B, seconds, n_steps=None, seed=0, conv_prec=None):
    cfg, m = _synth_model(name, seed)
    if conv_prec is not None:
        m._conv_prec = conv_prec
    mix = _clips(B, seconds, cfg["fs"], base=11)
    kw = {"n_steps": n_steps} if n_steps else {}
    with torch.no_grad():
        out = m.enhance(mix.to(DEV), rng=torch.Generator().manual_seed(20250614), **kw).cpu()
        ref = _oracle(m, cfg).enhance(mix, rng=torch.Generator().manual_seed(20250614), **kw)
    return m, out, ref


def test_c2_size_enhance_vs_oracle():
    """BASELINE configs[1]: PP16, one 8 s clip, 8 steps, default (split-f16)
    operands, against the fp32 oracle on the same noise."""
    m, out, ref = _vs_oracle("pp16", 1, 8.0)
    assert m._get_engine().conv_prec == 1
    assert out.shape == ref.shape == (1, 128000)
    assert rel_rms(out, ref) < 1e-3 and si_sdr(out, ref) > 60


def test_c1_size_enhance_vs_oracle():
    """BASELINE configs[0]: PP16, one 4 s clip (the reference's CPU-only
    plumbing case), 8 steps, the HIP path against the fp32 oracle on the same
    noise."""
    m, out, ref = _vs_oracle("pp16", 1, 4.0)
    assert out.shape == ref.shape == (1, 64000)
    assert rel_rms(out, ref) < 1e-3 and si_sdr(out, ref) > 60


def test_c3_shape_enhance_vs_oracle():
    """BASELINE configs[2]: ORIG16 full width, batch 8, 60 steps (0.25 s clips
    so the oracle finishes in seconds)."""
    m, out, ref = _vs_oracle("orig16", 8, 0.25, n_steps=60)
    assert out.shape == ref.shape == (8, 4000)
    assert rel_rms(out, ref) < 1e-3 and si_sdr(out, ref) > 60


def test_c4_shape_enhance_vs_oracle():
    """BASELINE configs[3]: PP24 full width (GRU H = 384), batch 4, 0.5 s
    clips, on the undamped synthetic weights, against the fp32 oracle on the
    same noise.  Their activations leave the split-f16 range at the default
    2^-6 staging exponent: the flagged layers' exponents widen (at most three
    reruns) and the result is still computed on split-f16 operands, with no
    f32 fallback."""
    m, out, ref = _vs_oracle("pp24", 4, 0.5)
    assert m._get_engine().conv_prec == 1 and m.range_fallbacks == 0
    assert m.range_widenings <= 3
    assert out.shape == ref.shape == (4, 12000)
    assert rel_rms(out, ref) < 1e-3 and si_sdr(out, ref) > 60


def test_c5_size_f16_enhance_vs_oracle():
    """BASELINE configs[4]: PP16, one 60 s clip, f16 conv operands, against the
    fp32 oracle: SI-SDR >= 30 dB, and the f16 path itself produced it."""
    m, out, ref = _vs_oracle("pp16", 1, 60.0, conv_prec=2)
    eng = m._get_engine()
    assert eng.conv_prec == 2 and int(eng.status.abs().sum()) == 0
    assert out.shape == ref.shape == (1, 960000)
    assert torch.isfinite(out).all() and si_sdr(out, ref) > 30


# ------------------------------------------------ queued / variable lengths
def test_enhance_many_equals_sequential_enhance():
    """Two clips in flight on two streams (Universe.enhance_many) give exactly
    the sequential enhance() results on the same noise sequence, for clips of
    different lengths."""
    d, cfg, m = _golden_model("pp16_c4", "pp16", 4)
    clips = [_t(synth_audio(n, 16000, i)[0]).to(DEV) for i, n in enumerate((4000, 5200, 4000, 3333, 5200))]
    with torch.no_grad():
        seq = [m.enhance(c, rng=g).cpu() for g in [torch.Generator().manual_seed(5)] for c in clips]
        many = [x.cpu() for x in m.enhance_many(clips, rng=torch.Generator().manual_seed(5), streams=2)]
    for a, b in zip(seq, many):
        assert a.shape == b.shape and torch.equal(a, b)


def test_variable_lengths_bounded_plans_and_memory(monkeypatch):
    """A stream of clips of distinct lengths (the CLI over a folder): tiles
    are tuned once per geometry (no new tuning for new lengths), the plan LRU
    stays bounded, and a second pass over the same lengths (every plan evicted
    and re-recorded) allocates no more device memory than the first."""
    monkeypatch.setenv("OUHIP_MAX_PLANS", "3")
    cfg, m = _synth_model("pp16")
    from open_universe_amd import engine as E

    lengths = [19000, 16000, 23000, 17500, 21000, 24500] * 2   # six distinct lengths, twice
    peaks = []
    with torch.no_grad():
        for i, n in enumerate(lengths):
            out = m.enhance(_t(synth_audio(n, 16000, i)[0]).to(DEV), rng=torch.Generator().manual_seed(i))
            assert out.shape == (n,) and torch.isfinite(out).all()
            if i == 0:
                timed = E._TUNER.timed
            torch.cuda.synchronize()
            peaks.append(torch.cuda.memory_allocated())
    assert len(m._plans) <= 3
    # later lengths reuse the first clip's tiles (new octave buckets copy them)
    assert E._TUNER.timed == timed
    assert max(peaks[6:]) <= max(peaks[:6]) * 1.05
