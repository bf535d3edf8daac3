from .norm import denormalize_batch, normalize_batch
from .stats import signal_median

__all__ = ["normalize_batch", "denormalize_batch", "signal_median"]
