"""Ensemble statistics (mirrors utils/stats.py:22-66)."""
import torch


def signal_median(signal):
    """Pick, per batch item, the ensemble member that is the sample-wise median
    most often.  signal: (ensemble, batch, ...) -> (batch, ...)."""
    shape = signal.shape
    signal = signal.flatten(start_dim=2)
    n = signal.shape[0]
    _, sorted_indices = signal.sort(dim=0)
    _, min_indices = abs(sorted_indices - n / 2).min(dim=0)
    pad_bins = torch.broadcast_to(torch.arange(n, device=signal.device)[None, :],
                                  (min_indices.shape[0], n))
    min_indices = torch.cat((min_indices, pad_bins), dim=1)
    counts = torch.cat([(min_indices == i).sum(dim=1, keepdim=True) for i in range(n)], dim=1) - 1
    select = counts.argmax(dim=1)
    median_signal = torch.stack([signal[select[i], i, :] for i in range(signal.shape[1])], dim=0)
    return median_signal.reshape(shape[1:])
