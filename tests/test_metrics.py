"""F3/F4 host side (CPU): the metric restatements (SI-SDR, LSD, SI-LSD) on
known answers, the STFT convention against a direct DFT, WAV I/O, the
evaluation CLI, and the resampling table against the oracle's restatement of
torchaudio's kernel."""
import json
import math

import numpy as np
import pytest
import torch

from open_universe_amd import dsp, metrics
from open_universe_amd.audio import load_audio, save_audio
from open_universe_amd.bin import eval_metrics
from oracle import ou_oracle as O


def _sig(n=16000, seed=0):
    g = torch.Generator().manual_seed(seed)
    t = torch.arange(n, dtype=torch.float64) / 16000
    return torch.sin(2 * math.pi * 440 * t) + 0.1 * torch.randn(n, generator=g, dtype=torch.float64)


def test_si_sdr_known_answers():
    r = _sig()
    g = torch.Generator().manual_seed(1)
    n = torch.randn(r.shape, generator=g, dtype=torch.float64)
    n = n - (n @ r) / (r @ r) * r          # orthogonal to r
    n = n * (r.norm() / n.norm()) * 10 ** (-15 / 20)   # 15 dB below r
    for scale in (1.0, 0.3, -2.0):         # scale invariant, sign included
        assert float(metrics.si_sdr(r, scale * (r + n))) == pytest.approx(15.0, abs=1e-9)
    assert float(metrics.si_sdr(r, 3 * r)) == pytest.approx(100.0)     # clamp_db
    assert float(metrics.si_sdr(r, n)) == pytest.approx(-100.0)        # orthogonal -> -clamp
    b = metrics.si_sdr(torch.stack([r, r]), torch.stack([r + n, 2 * (r + n)]))
    assert b.shape == (2,) and torch.allclose(b, torch.full((2,), 15.0, dtype=torch.float64))


def test_lsd_known_answers():
    r = _sig().float()
    assert float(metrics.lsd(r, r)) == pytest.approx(0.0, abs=1e-9)
    # a gain g shifts every bin by 20 log10 g dB (up to the eps = 1e-7 floor)
    assert float(metrics.lsd(r, 2 * r)) == pytest.approx(20 * math.log10(2), rel=2e-4)
    # the reference's SI-LSD rescales the target by <deg, ref> / <deg, deg>
    # (lsd.py:96-99), so deg = 0.5 ref gives ref' = 2 ref: 20 log10(4) dB
    assert float(metrics.si_lsd(r, 0.5 * r)) == pytest.approx(20 * math.log10(4), rel=2e-4)
    # 24 kHz: 25 ms / 10 ms frames at that rate
    r24 = _sig(24000).float()
    assert float(metrics.lsd(r24, 2 * r24, fs=24000)) == pytest.approx(20 * math.log10(2), rel=2e-4)


def test_power_spec_is_torchaudio_spectrogram_convention():
    """centered frames, reflect padding, periodic Hann, power 2, divided by the
    window's L2 norm (torchaudio.functional.spectrogram, normalized='window')."""
    n_fft, hop = 16, 4
    x = _sig(50, seed=3)
    w = torch.hann_window(n_fft, periodic=True, dtype=torch.float64)
    got = metrics._power_spec(x, n_fft, hop, w).numpy()
    xp = np.pad(x.numpy(), n_fft // 2, mode="reflect")
    frames = np.stack([xp[i * hop:i * hop + n_fft] for i in range(1 + len(x) // hop)], 1)
    spec = np.fft.rfft(frames * w.numpy()[:, None], axis=0) / np.sqrt((w.numpy() ** 2).sum())
    np.testing.assert_allclose(got, np.abs(spec) ** 2, rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("dtype", [np.int16, np.int32, np.float32])
def test_wav_roundtrip(tmp_path, dtype):
    from scipy.io import wavfile

    rng = np.random.default_rng(0)
    if dtype == np.float32:
        a = rng.uniform(-1, 1, (1000, 2)).astype(np.float32)
        want = a.T
    else:
        info = np.iinfo(dtype)
        a = rng.integers(info.min, info.max, (1000, 2), dtype=dtype)
        want = a.T.astype(np.float64) / -float(info.min)
    wavfile.write(tmp_path / "a.wav", 22050, a)
    x, fs = load_audio(tmp_path / "a.wav")
    assert fs == 22050 and x.shape == (2, 1000) and x.dtype == torch.float32
    np.testing.assert_allclose(x.numpy(), want, rtol=1e-6, atol=1e-7)
    save_audio(tmp_path / "b.wav", x, fs)
    y, fs2 = load_audio(tmp_path / "b.wav")
    assert fs2 == fs and torch.equal(x, y)
    save_audio(tmp_path / "m.wav", x[0], fs)          # (T,) -> mono
    m, _ = load_audio(tmp_path / "m.wav")
    assert m.shape == (1, 1000) and torch.equal(m[0], x[0])


def test_eval_metrics_cli(tmp_path):
    ref_dir, deg_dir = tmp_path / "ref", tmp_path / "deg"
    ref_dir.mkdir()
    (deg_dir / "sub").mkdir(parents=True)
    r = _sig().float()
    save_audio(ref_dir / "a.wav", r, 16000)
    save_audio(ref_dir / "b.wav", r, 16000)
    save_audio(deg_dir / "a.wav", 2 * r, 16000)
    save_audio(deg_dir / "sub" / "b.wav", torch.cat([r, r[:100]]), 16000)   # longer: cropped
    save_audio(deg_dir / "orphan.wav", r, 16000)                           # no reference: skipped
    out = tmp_path / "res.json"
    assert eval_metrics.main([str(deg_dir), "--ref", str(ref_dir), "--result", str(out)]) == 0
    res = json.loads(out.read_text())
    assert set(res["files"]) == {"a", "b"} and res["summary"]["number"] == 2
    assert res["files"]["a"]["si-sdr"] == pytest.approx(100.0)
    assert res["files"]["a"]["lsd"] == pytest.approx(20 * math.log10(2), rel=2e-4)
    assert res["files"]["b"]["lsd"] == pytest.approx(0.0, abs=1e-6)
    assert res["summary"]["lsd"] == pytest.approx(10 * math.log10(2), rel=2e-4)


def test_summarize_matches_reference_semantics():
    s = eval_metrics.summarize({"a": {"x": 1.0, "y": "skip"}, "b": {"x": 3.0}})
    assert s == {"x": 2.0, "number": 2}


@pytest.mark.parametrize("orig,new", [(48000, 16000), (16000, 24000), (44100, 16000), (22050, 16000),
                                      (8000, 16000), (1, 2), (2, 1)])
def test_resample_table_matches_oracle(orig, new):
    k, width = dsp.sinc_resample_kernel(orig, new)
    ko, wo, o, n = O._sinc_resample_kernel(orig, new)
    assert width == wo and k.shape == (n, 2 * width + o)
    np.testing.assert_array_equal(k, ko.reshape(n, -1).numpy())


def test_lsd_and_si_lsd_vs_reference_fixtures():
    """F4 pinned to the reference: tests/golden/metrics.npz holds the outputs
    of the reference's own log_spectral_distance (metrics/lsd.py:26-140, loaded
    by path in make_golden.py; torchaudio.functional.spectrogram restated) with
    the wrapper's 25 ms / 10 ms frames (metrics/wrapper.py:130-151) on random,
    rescaled and enhanced-vs-clean pairs at 16 and 24 kHz.  The restatement
    computes in float64: equal to the float64 reference to 1e-9, and to the
    float32 reference (the dtype the reference keeps) to 1e-4 relative."""
    from conftest import load_golden

    d = load_golden("metrics")
    keys = sorted({k.rsplit("_", 1)[0] for k in d if k.endswith("_ref")})
    assert len(keys) == 5
    for key in keys:
        fs = int(key.split("_")[0][2:])
        ref, deg = torch.from_numpy(d[f"{key}_ref"]), torch.from_numpy(d[f"{key}_deg"])
        got = metrics.lsd(ref, deg, fs=fs).numpy()
        got_si = metrics.si_lsd(ref, deg, fs=fs).numpy()
        np.testing.assert_allclose(got, d[f"{key}_lsd_f64"], rtol=1e-9, err_msg=key)
        np.testing.assert_allclose(got_si, d[f"{key}_silsd_f64"], rtol=1e-9, err_msg=key)
        np.testing.assert_allclose(got, d[f"{key}_lsd_f32"], rtol=1e-4, err_msg=key)
        np.testing.assert_allclose(got_si, d[f"{key}_silsd_f32"], rtol=1e-4, err_msg=key)
