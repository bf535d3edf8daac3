"""Ensemble reductions on the device (Universe.enhance's ``ensemble_stat``,
reference networks/universe/universe.py:359-368 and utils/stats.py:22-66).

Each call launches the HIP kernels through the C ABI (``ou_ensemble_reduce``
for mean / median, ``ou_signal_median`` for signal_median) on the current
stream; there is no host or ATen fallback.  ``signal_median``'s selection rule
is documented on the kernel (csrc/ou_misc.hip).
"""
import torch

from .. import _lib as L

_MODES = {"mean": 0, "median": 1}


def _check(x):
    if x.device.type != "cuda":
        raise L.OuHipError("ensemble reductions run on the HIP device")
    if x.shape[0] > 32:
        raise ValueError("at most 32 ensemble members")
    return x.to(torch.float32).contiguous()


def signal_median(signal):
    """(E, B, ...) -> (B, ...): per batch item, the member chosen by the
    reference's per-sample rank vote."""
    x = _check(signal)
    E, B = x.shape[0], x.shape[1]
    n = x[0, 0].numel()
    y = torch.empty(x.shape[1:], dtype=torch.float32, device=x.device)
    counts = torch.empty((B, 32), dtype=torch.int32, device=x.device)
    stream = torch.cuda.current_stream(x.device).cuda_stream
    L.check(L.load().ou_signal_median(x.data_ptr(), y.data_ptr(), E, B, n, counts.data_ptr(), stream),
            "signal_median")
    return y


def ensemble_reduce(x, stat):
    """x: (E, B, ...) -> (B, ...) for ensemble_stat in {mean, median,
    signal_median}."""
    if stat == "signal_median":
        return signal_median(x)
    if stat not in _MODES:
        raise NotImplementedError()
    x = _check(x)
    y = torch.empty(x.shape[1:], dtype=torch.float32, device=x.device)
    stream = torch.cuda.current_stream(x.device).cuda_stream
    L.check(L.load().ou_ensemble_reduce(x.data_ptr(), y.data_ptr(), x.shape[0], y.numel(), _MODES[stat], stream),
            "ensemble_reduce")
    return y
