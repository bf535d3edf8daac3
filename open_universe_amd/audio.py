"""Audio I/O and resampling around ``enhance()``.

The reference CLI reads files with ``torchaudio.load``, resamples with
``torchaudio.functional.resample`` to ``model.fs`` and back, and writes with
``torchaudio.save`` (bin/enhance.py:61-64, 183-192).  Here:

* ``resample`` runs on the GPU (``ou_resample``, csrc/ou_audio.hip) with
  torchaudio's default polyphase windowed-sinc table (``dsp.sinc_resample_kernel``);
* ``load_audio`` / ``save_audio`` read and write WAV (torchaudio is not in this
  image; mp3/flac decoding is out of scope) with torchaudio's normalisation of
  integer PCM to float32 in [-1, 1).
"""
import math

import numpy as np
import torch

from . import _lib as L
from . import dsp

_KERNELS = {}


def _kernel(orig, new, device):
    g = math.gcd(orig, new)
    key = (orig // g, new // g, str(device))
    if key not in _KERNELS:
        k, width = dsp.sinc_resample_kernel(orig // g, new // g)
        _KERNELS[key] = (torch.from_numpy(np.ascontiguousarray(k)).to(device), width)
    return key[0], key[1], _KERNELS[key]


def resample(x: torch.Tensor, orig_freq: int, new_freq: int) -> torch.Tensor:
    """torchaudio.functional.resample(x, orig_freq, new_freq) on a ROCm
    device tensor (..., T); same output length ceil(new * T / orig)."""
    if orig_freq == new_freq:
        return x
    if not x.is_cuda:
        raise L.OuHipError("resample: the HIP path needs a ROCm device tensor")
    o, n, (k, width) = _kernel(int(orig_freq), int(new_freq), x.device)
    shape = x.shape
    xs = x.reshape(-1, shape[-1]).to(torch.float32).contiguous()
    n_in = xs.shape[-1]
    n_out = int(math.ceil(n * n_in / o))
    y = torch.empty(xs.shape[0], n_out, device=x.device, dtype=torch.float32)
    L.check(L.load().ou_resample(xs.data_ptr(), n_in, y.data_ptr(), n_out, xs.shape[0], n_in, n_out,
                                 k.data_ptr(), n, k.shape[1], o, width,
                                 torch.cuda.current_stream(x.device).cuda_stream), "resample")
    return y.reshape(shape[:-1] + (n_out,))


def load_audio(path):
    """(channels, frames) float32 tensor and the sample rate, as
    ``torchaudio.load(path)`` returns them for a WAV file."""
    from scipy.io import wavfile

    fs, data = wavfile.read(str(path))
    if data.dtype == np.int16:
        x = data.astype(np.float32) / 32768.0
    elif data.dtype == np.int32:
        x = data.astype(np.float32) / 2147483648.0
    elif data.dtype == np.uint8:
        x = (data.astype(np.float32) - 128.0) / 128.0
    else:
        x = data.astype(np.float32)
    x = x.reshape(x.shape[0], -1).T if x.ndim > 1 else x[None, :]
    return torch.from_numpy(np.ascontiguousarray(x)), int(fs)


def save_audio(path, x: torch.Tensor, fs: int):
    """Write (channels, frames) or (frames,) as a 32-bit float WAV (what
    ``torchaudio.save`` writes for a float32 tensor)."""
    from scipy.io import wavfile

    a = x.detach().to("cpu", torch.float32).numpy()
    if a.ndim == 2:
        a = a.T if a.shape[0] > 1 else a[0]
    wavfile.write(str(path), int(fs), np.ascontiguousarray(a, dtype=np.float32))
