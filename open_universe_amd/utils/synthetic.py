"""Deterministic synthetic weights and audio.

No trained checkpoint and no Voicebank-DEMAND audio exist offline, so tests,
golden fixtures and the benchmark all use weights generated from
``(parameter name, shape, seed)`` alone.  Because the generator only needs the
name and the shape, the reference model (golden fixtures, generated in the
build container) and this package (GPU box) get bit-identical weights without
shipping any weight file.

Scales are chosen so activations stay O(1) through the network: weight-normed
layers get ``g ~ 1`` (unit-norm rows, the reference's ``cond_weight_norm``,
``blocks.py:40-46``), plain layers get ``1/sqrt(fan_in)``.

The "damped" family (``rc_gain=RC_DAMP``) also scales ``g`` of every
rate-change conv: the binomial anti-alias FIRs are normalised to unit RMS, not
unit DC gain (``blocks.py:66-72``), so with ``g ~ 1`` each anti-aliased rate
change amplifies by 4-9x and the reference's own PP24 activations reach 7.7e6
(golden ``pp24.npz`` ``enh_peak_activation``), beyond what trained weights
produce and beyond the split-f16 operand range.  At ``RC_DAMP`` they stay O(10)
(``pp24d.npz``), the regime trained models run in.
"""
import math
import zlib

import numpy as np
import torch


def _gen(name, seed):
    g = torch.Generator()
    g.manual_seed((int(seed) * 1000003 + zlib.crc32(name.encode())) % (2**62))
    return g


RC_DAMP = 0.25   # rate-change conv weight_g scale of the damped family


def synth_tensor(name, shape, seed=0, rc_gain=1.0):
    """Synthetic value for one state-dict entry, or ``None`` for deterministic
    buffers that the module computes itself (FIR taps, mel filterbank, STFT
    window, resampling kernels).  ``rc_gain`` scales the weight-norm gain of
    the rate-change convs (the damped family, see the module doc)."""
    shape = tuple(int(s) for s in shape)
    g = _gen(name, seed)
    leaf = name.rsplit(".", 1)[-1]
    n = 1
    for s in shape:
        n *= s

    if leaf in ("weights", "window", "fb", "kernel"):
        return None  # deterministic buffers
    if leaf == "freq":  # SigmaBlock random Fourier features (sigma_block.py:43)
        return 16.0 * torch.randn(shape, generator=g)
    if name.endswith("sigma_block.weight"):  # SimpleTimeEmbedding (sigma_block.py:68)
        return 0.8 + 0.3 * torch.rand(shape, generator=g)
    if name.endswith("sigma_block.bias"):
        return 0.4 * torch.randn(shape, generator=g)
    if leaf == "alpha":  # Snake log-alpha (bigvgan/snake.py:44)
        return 0.3 * torch.randn(shape, generator=g)
    if leaf == "weight_g":
        v = 1.0 + 0.2 * (2.0 * torch.rand(shape, generator=g) - 1.0)
        return v * rc_gain if (rc_gain != 1.0 and "rate_change_conv" in name) else v
    if leaf == "weight_v":
        return torch.randn(shape, generator=g)
    if "prelu" in name and leaf == "weight" and n == 1:
        return 0.05 + 0.4 * torch.rand(shape, generator=g)
    if leaf.startswith("weight_") or leaf.startswith("bias_"):  # torch GRU
        # weight_ih_l0 (3H, I), weight_hh_l0 (3H, H), bias_* (3H,)
        hidden = shape[0] // 3
        k = 1.0 / math.sqrt(hidden)
        return k * (2.0 * torch.rand(shape, generator=g) - 1.0)
    if leaf == "bias":
        return 0.1 * torch.randn(shape, generator=g)
    if leaf == "weight":
        fan_in = 1
        for s in shape[1:]:
            fan_in *= s
        return torch.randn(shape, generator=g) / math.sqrt(max(fan_in, 1))
    return 0.1 * torch.randn(shape, generator=g)


def fill_module_(module, seed=0, skip_prefixes=("loss_",), rc_gain=1.0):
    """Overwrite a module's parameters/buffers in place with synthetic values."""
    sd = module.state_dict()
    new = {}
    for name, t in sd.items():
        if name.startswith(tuple(skip_prefixes)):
            continue
        v = synth_tensor(name, t.shape, seed, rc_gain)
        if v is not None:
            new[name] = v.to(t.dtype)
    module.load_state_dict(new, strict=False)
    return module


def synth_state_dict(spec, seed=0, rc_gain=1.0):
    """spec: iterable of (name, shape) -> {name: tensor} (deterministic buffers
    are omitted; the consumer recomputes them)."""
    out = {}
    for name, shape in spec:
        v = synth_tensor(name, shape, seed, rc_gain)
        if v is not None:
            out[name] = v
    return out


def synth_audio(n_samples, fs=16000, index=0, snr_db=5.0):
    """Synthetic noisy speech-like clip.

    White noise plus a harmonic stack (f0 ~ U(100, 250) Hz, 10 harmonics, 1/k
    amplitudes, 4 Hz AM envelope) mixed at ``snr_db``; float32 numpy array.
    """
    rng = np.random.default_rng(20250614 + index)
    t = np.arange(n_samples) / fs
    f0 = rng.uniform(100.0, 250.0)
    phases = rng.uniform(0, 2 * np.pi, size=10)
    harm = np.zeros(n_samples)
    for k in range(1, 11):
        if k * f0 < fs / 2:
            harm += np.sin(2 * np.pi * k * f0 * t + phases[k - 1]) / k
    env = 0.6 + 0.4 * np.sin(2 * np.pi * 4.0 * t + rng.uniform(0, 2 * np.pi))
    clean = harm * env
    noise = rng.standard_normal(n_samples)
    p_c = np.mean(clean**2)
    p_n = np.mean(noise**2)
    noise *= math.sqrt(p_c / (p_n * 10 ** (snr_db / 10.0)))
    mix = 0.1 * (clean + noise) / math.sqrt(p_c)
    return mix.astype(np.float32), (0.1 * clean / math.sqrt(p_c)).astype(np.float32)
