"""Amplitude normalisation (mirrors utils/norm.py:22-91).

On the enhance() path this runs as the ``ou_normalize`` kernel; this tensor
version serves the sampler known-answer mode and API parity.
"""
import torch


def _norm2(signal, eps=1e-5):
    return signal.std(dim=(1, 2), keepdim=True).clamp(min=eps)


def _norm_max(signal, eps=1e-5):
    std = abs(signal.view((signal.shape[0], -1))).max(dim=1).values
    return std[:, None, None].clamp(min=eps)


def _compute_gain(signal, norm, level, eps=1e-5):
    if norm == 2 or norm == "2":
        return level / _norm2(signal)
    if norm == "max":
        return level / _norm_max(signal)
    if norm == "2-max":
        return torch.minimum(level / _norm2(signal, eps=eps), 1.0 / _norm_max(signal, eps=eps))
    raise NotImplementedError(f"Norm {norm} is not implemented for batch normalization")


def normalize_batch(batch, norm=2, level_db=0.0, ref="noisy", eps=1e-5, zero_mean=True):
    assert ref in ["noisy", "both"]
    level = 10 ** (level_db / 20.0)
    mix, *others = batch
    if zero_mean:
        mean = mix.mean(dim=(1, 2), keepdim=True)
        mix = mix - mean
    else:
        mean = 0.0
    gain = _compute_gain(mix, norm, level, eps=eps)
    mix = mix * gain
    out = [mix]
    for tgt in others:
        if tgt is not None:
            if ref == "both":
                if zero_mean:
                    tgt = tgt - tgt.mean(dim=(1, 2), keepdim=True)
                tgt = tgt * _compute_gain(tgt, norm, level, eps=eps)
            else:
                tgt = (tgt - mean) * gain
        out.append(tgt)
    return out, mean, 1.0 / gain


def denormalize_batch(x, mean, std):
    return x * std + mean
