"""Batch level normalisation (reference utils/norm.py:47-91, ``norm=2``).

On the enhance() path this is the ``ou_normalize`` kernel.  This tensor form
serves only the sampler known-answer mode (``enhance(target=...)``), whose
arithmetic is tensor ops by design; ``Universe`` accepts ``norm=2`` only, so
the ``"max"`` / ``"2-max"`` norms are not restated.
"""
import torch


def _centre_and_gain(x, level, eps, zero_mean):
    """Per item over (channels, samples): the mean that is removed and the gain
    level / max(std, eps), with torch's unbiased std of the centred signal."""
    mu = x.mean(dim=(1, 2), keepdim=True) if zero_mean else torch.zeros_like(x[:, :1, :1])
    gain = level / (x - mu).std(dim=(1, 2), keepdim=True).clamp(min=eps)
    return mu, gain


def normalize_batch(batch, norm=2, level_db=0.0, ref="noisy", eps=1e-5, zero_mean=True):
    """Normalise ``batch = (mix, *targets)`` to ``level_db``.  ``ref="both"``
    normalises every target on its own statistics, ``ref="noisy"`` applies the
    mixture's.  Returns ``([mix, *targets], mean, 1 / gain)``."""
    if str(norm) != "2":
        raise NotImplementedError(f"Norm {norm} is not implemented for batch normalization")
    if ref not in ("noisy", "both"):
        raise ValueError(f"ref must be 'noisy' or 'both', got {ref!r}")
    level = 10.0 ** (level_db / 20.0)
    mix, *targets = batch
    mu, gain = _centre_and_gain(mix, level, eps, zero_mean)
    out = [(mix - mu) * gain]
    for t in targets:
        if t is not None:
            tm, tg = _centre_and_gain(t, level, eps, zero_mean) if ref == "both" else (mu, gain)
            t = (t - tm) * tg
        out.append(t)
    return out, (mu if zero_mean else 0.0), 1.0 / gain


def denormalize_batch(x, mean, std):
    return x * std + mean
