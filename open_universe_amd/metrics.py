"""Quality metrics of the enhance() output.

Restates the reference's evaluation wrapper (metrics/wrapper.py:95-213,
metrics/lsd.py:26-140) for the metrics computable offline:

* ``si_sdr`` -- fast_bss_eval.si_sdr(ref, deg, zero_mean=False, clamp_db=100)
  (wrapper.py:197-213): the closed form with the projection of the estimate
  on the reference, clamped to [-100, 100] dB;
* ``lsd`` / ``si_lsd`` -- log_spectral_distance (lsd.py:26-140) with its
  defaults scaled to the sample rate (25 ms window, 10 ms hop, wrapper.py
  lsd()), on torch.stft with torchaudio.functional.spectrogram's semantics
  (centered, reflect padding, power 2, normalized="window");
* ``pesq_wb`` -- ITU-T P.862.2 through the ``pesq`` package when importable.
  It is not in this image, so PESQ parity is unpinned here.

All functions take (..., T) tensors on any device and compute in float64.
"""
import math

import torch


def si_sdr(ref: torch.Tensor, deg: torch.Tensor, clamp_db: float = 100.0) -> torch.Tensor:
    """Scale-invariant SDR in dB, per signal (fast_bss_eval, zero_mean=False)."""
    r = ref.to(torch.float64)
    d = deg.to(torch.float64)
    alpha = (r * d).sum(-1, keepdim=True) / (r * r).sum(-1, keepdim=True)
    t = alpha * r
    num = (t * t).sum(-1)
    den = ((d - t) ** 2).sum(-1)
    ratio = num / den
    # clamp the ratio to [10^(-clamp/10), 10^(clamp/10)] before the log
    lim = 10.0 ** (clamp_db / 10.0)
    ratio = torch.nan_to_num(ratio, nan=lim, posinf=lim).clamp(1.0 / lim, lim)
    return 10.0 * torch.log10(ratio)


def _power_spec(x, n_fft, hop, window):
    # torchaudio.functional.spectrogram(pad=0, power=2, normalized="window",
    # center=True, pad_mode="reflect", onesided=True)
    shape = x.shape
    s = torch.stft(x.reshape(-1, shape[-1]), n_fft=n_fft, hop_length=hop, win_length=n_fft, window=window,
                   center=True, pad_mode="reflect", normalized=False, onesided=True, return_complex=True)
    s = s / window.pow(2.0).sum().sqrt()
    p = s.abs().pow(2.0)
    return p.reshape(shape[:-1] + p.shape[-2:])


def lsd(ref: torch.Tensor, deg: torch.Tensor, fs: int = 16000, scale_invariant: bool = False,
        p: float = 2.0, eps: float = 1e-7) -> torch.Tensor:
    """Log-spectral distance in dB (lsd.py:26-140; n_fft = 25 ms, hop = 10 ms
    at ``fs`` as in wrapper.py lsd())."""
    n_fft = int(0.025 * fs)
    hop = int(0.01 * fs)
    x = deg.to(torch.float64)
    t = ref.to(torch.float64)
    window = torch.hann_window(n_fft, periodic=True, dtype=torch.float64, device=x.device)
    if scale_invariant:
        t = t * ((x * t).sum(-1, keepdim=True) / ((x * x).sum(-1, keepdim=True) + eps))
    a = 10.0 * torch.log10(_power_spec(x, n_fft, hop, window) + eps)
    b = 10.0 * torch.log10(_power_spec(t, n_fft, hop, window) + eps)
    denom = (b.shape[-1] * b.shape[-2]) ** (1.0 / p)
    return torch.linalg.vector_norm(a - b, ord=p, dim=(-2, -1)) / denom


def si_lsd(ref, deg, fs=16000):
    return lsd(ref, deg, fs, scale_invariant=True)


def pesq_wb(ref: torch.Tensor, deg: torch.Tensor, fs: int = 16000) -> float:
    """PESQ-wb at 16 kHz (wrapper.py:95-108).  Needs the ``pesq`` package."""
    try:
        from pesq import pesq
    except ImportError as e:   # not in this image
        raise NotImplementedError("PESQ needs the `pesq` package (ITU-T P.862 C code), not installed") from e
    if fs != 16000:
        from .audio import resample

        ref, deg = resample(ref, fs, 16000), resample(deg, fs, 16000)
    return float(pesq(16000, ref.cpu().double().numpy(), deg.cpu().double().numpy(), "wb"))


METRICS = {"si-sdr": lambda r, d, fs: float(si_sdr(r, d).mean()),
           "lsd": lambda r, d, fs: float(lsd(r, d, fs).mean()),
           "si-lsd": lambda r, d, fs: float(si_lsd(r, d, fs).mean())}
