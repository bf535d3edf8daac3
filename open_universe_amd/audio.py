"""Audio I/O and resampling around ``enhance()``.

The reference CLI reads files with ``torchaudio.load``, resamples with
``torchaudio.functional.resample`` to ``model.fs`` and back, and writes with
``torchaudio.save`` (bin/enhance.py:61-64, 183-192).  Here:

* ``resample`` runs on the GPU (``ou_resample``, csrc/ou_audio.hip) with
  torchaudio's default polyphase windowed-sinc table (``dsp.sinc_resample_kernel``);
* ``load_audio`` reads WAV (scipy) and FLAC (``ou_flac_decode``, a native
  decoder in csrc/ou_flac.cpp: libFLAC and torchaudio are not in this image)
  with torchaudio's normalisation of integer PCM to float32 in [-1, 1);
  ``save_audio`` writes WAV, or 24-bit FLAC for a .flac path (``ou_flac_encode``).
  mp3 stays out of scope (no decoder here).
"""
import ctypes
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


def load_flac(path):
    """(channels, frames) float32 tensor and the sample rate of a FLAC file,
    scaled as ``torchaudio.load`` scales integer PCM (sample / 2^(bps-1))."""
    lib = L.load()
    with open(path, "rb") as fh:
        data = fh.read()
    buf = ctypes.create_string_buffer(data, len(data))
    fs, ch, bps, n = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
    L.check(lib.ou_flac_info(buf, len(data), ctypes.byref(fs), ctypes.byref(ch), ctypes.byref(bps),
                             ctypes.byref(n)), f"flac {path}")
    out = np.zeros((ch.value, n.value), dtype=np.float32)
    got = lib.ou_flac_decode(buf, len(data), out.ctypes.data, n.value)
    if got < 0:
        L.check(int(got), f"flac {path}")
    if got != n.value:
        raise L.OuHipError(f"flac {path}: decoded {got} frames, STREAMINFO says {n.value}")
    return torch.from_numpy(out), int(fs.value)


def audio_info(path):
    """(channels, frames, sample rate) of a WAV or FLAC file without decoding
    it (torchaudio.info's num_channels / num_frames / sample_rate)."""
    if str(path).lower().endswith(".flac"):
        lib = L.load()
        with open(path, "rb") as fh:
            data = fh.read()
        buf = ctypes.create_string_buffer(data, len(data))
        fs, ch, bps, n = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
        L.check(lib.ou_flac_info(buf, len(data), ctypes.byref(fs), ctypes.byref(ch), ctypes.byref(bps),
                                 ctypes.byref(n)), f"flac {path}")
        return int(ch.value), int(n.value), int(fs.value)
    return _wav_info(path)


def _wav_info(path):
    """(channels, frames, sample rate) from a WAV file's RIFF 'fmt ' and
    'data' chunk headers: frames = data bytes // block align.  Reads headers
    only, so every container width works (scipy's mmap reader refuses 24-bit
    PCM, which ``load_audio`` reads)."""
    import os
    import struct

    size = os.path.getsize(path)
    with open(path, "rb") as fh:
        head = fh.read(12)
        if len(head) < 12 or head[:4] != b"RIFF" or head[8:12] != b"WAVE":
            raise ValueError(f"{path}: not a RIFF/WAVE file")
        ch = fs = align = None
        while True:
            hdr = fh.read(8)
            if len(hdr) < 8:
                raise ValueError(f"{path}: no 'data' chunk")
            cid, n = hdr[:4], struct.unpack("<I", hdr[4:])[0]
            if cid == b"fmt ":
                fmt = fh.read(n)
                if len(fmt) < 16:
                    raise ValueError(f"{path}: short 'fmt ' chunk")
                _, ch, fs, _, align = struct.unpack("<HHIIH", fmt[:14])
                if n & 1:
                    fh.seek(1, 1)
            elif cid == b"data":
                if ch is None or not align:
                    raise ValueError(f"{path}: 'data' before 'fmt '")
                n = min(n, size - fh.tell())   # streamed files may carry 0xFFFFFFFF
                return int(ch), int(n // align), int(fs)
            else:
                fh.seek(n + (n & 1), 1)


def resampled_len(n, orig_freq, new_freq):
    """Output length of ``resample`` (ceil(new * n / orig) in lowest terms)."""
    if orig_freq == new_freq:
        return n
    g = math.gcd(int(orig_freq), int(new_freq))
    return int(math.ceil((new_freq // g) * n / (orig_freq // g)))


def load_audio(path):
    """(channels, frames) float32 tensor and the sample rate, as
    ``torchaudio.load(path)`` returns them for a WAV or FLAC file."""
    from scipy.io import wavfile

    if str(path).lower().endswith(".flac"):
        return load_flac(path)

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


def save_flac(path, x: torch.Tensor, fs: int, bits: int = 24):
    """Write (channels, frames) or (frames,) as a FLAC file of ``bits``-bit
    PCM (``ou_flac_encode``)."""
    lib = L.load()
    a = x.detach().to("cpu", torch.float32).numpy()
    a = np.ascontiguousarray(a[None] if a.ndim == 1 else a)
    ch, n = a.shape
    cap = lib.ou_flac_encode_bound(ch, n, bits)
    buf = (ctypes.c_uint8 * cap)()
    got = lib.ou_flac_encode(a.ctypes.data, ch, n, int(fs), bits, buf, cap)
    if got < 0:
        L.check(int(got), f"flac {path}")
    with open(path, "wb") as fh:
        fh.write(bytes(buf)[:got])


def save_audio(path, x: torch.Tensor, fs: int):
    """Write (channels, frames) or (frames,): a 32-bit float WAV (what
    ``torchaudio.save`` writes for a float32 tensor), or 24-bit FLAC for a
    ``.flac`` path."""
    from scipy.io import wavfile

    if str(path).lower().endswith(".flac"):
        return save_flac(path, x, fs)
    a = x.detach().to("cpu", torch.float32).numpy()
    if a.ndim == 2:
        a = a.T if a.shape[0] > 1 else a[0]
    wavfile.write(str(path), int(fs), np.ascontiguousarray(a, dtype=np.float32))
