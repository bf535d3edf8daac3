"""Deterministic signal-processing constants of the hot path.

These are the buffers the reference builds at construction time (and stores
in its checkpoints): binomial anti-alias taps, the STFT window, the mel
filterbank and the sinc resampling kernels of the alias-free Snake.  They are
recomputed here (numpy, float64 then cast) so the product path never depends
on the test oracle.
"""
import math

import numpy as np


def binomial_taps(kernel_size):
    """Unit-RMS binomial FIR (networks/universe/blocks.py:66-72).  Pascal row
    k-1 normalised by the RMS of the whole Pascal matrix, cast to float32, then
    renormalised to unit RMS in float32 -- reproduced step for step."""
    n = kernel_size
    pascal = np.zeros((n, n), dtype=np.float64)
    for i in range(n):
        for j in range(i + 1):
            pascal[i, j] = math.comb(i, j)
    norm = np.sqrt(np.mean(pascal**2))
    taps = (pascal[n - 1, :] / norm).astype(np.float32)
    rms = np.sqrt(np.mean(np.square(taps, dtype=np.float32), dtype=np.float32), dtype=np.float32)
    return (taps / rms).astype(np.float32)


def hann_periodic(n):
    """torch.hann_window(n, periodic=True): the window torchaudio's Spectrogram
    multiplies each frame by (bit-identical float32 values)."""
    import torch

    return torch.hann_window(n).numpy().astype(np.float32)


def melscale_fbanks(n_freqs, f_min, f_max, n_mels, sample_rate):
    """HTK mel filterbank with norm=None (torchaudio.functional.melscale_fbanks
    semantics, which MelAdapter uses with sample_rate hard-coded to 24000:
    networks/universe/condition.py:75-81).  Evaluated with float32 torch CPU
    ops in torchaudio's order so the table is bit-identical to the buffer a
    reference checkpoint stores."""
    import torch

    all_freqs = torch.linspace(0, sample_rate // 2, n_freqs)
    m_min = 2595.0 * math.log10(1.0 + f_min / 700.0)
    m_max = 2595.0 * math.log10(1.0 + f_max / 700.0)
    m_pts = torch.linspace(m_min, m_max, n_mels + 2)
    f_pts = 700.0 * (10.0 ** (m_pts / 2595.0) - 1.0)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
    down = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    fb = torch.max(torch.zeros(1), torch.min(down, up))
    return fb.numpy().astype(np.float32)


def sinc_resample_kernel(orig, new, lowpass_width=6, rolloff=0.99):
    """Windowed-sinc (Hann) polyphase kernel of torchaudio's
    Resample(resampling_method='sinc_interp_hann'), used by the alias-free Snake
    (networks/bigvgan/alias_free_act.py:17-18).  Returns (kernel[new][taps],
    width) with taps = 2*width + orig."""
    g = math.gcd(orig, new)
    orig, new = orig // g, new // g
    base = min(orig, new) * rolloff
    width = math.ceil(lowpass_width * orig / base)
    idx = np.arange(-width, width + orig, dtype=np.float64)[None, :] / orig
    t = (np.arange(0, -new, -1, dtype=np.float32)[:, None] / np.float32(new)).astype(np.float64) + idx
    t = t * base
    t = np.clip(t, -lowpass_width, lowpass_width)
    window = np.cos(t * math.pi / lowpass_width / 2) ** 2
    t = t * math.pi
    scale = base / orig
    with np.errstate(invalid="ignore", divide="ignore"):
        k = np.where(t == 0, 1.0, np.sin(t) / t)
    k = k * window * scale
    return k.astype(np.float32), width
