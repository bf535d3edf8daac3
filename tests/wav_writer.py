"""Test helper: PCM WAV files in container widths scipy.io.wavfile.write does
not produce (24-bit), written from the RIFF layout directly."""
import struct

import numpy as np


def write_wav24(path, fs, x, extra_chunk=True):
    """x: float array (frames,) or (frames, channels) in [-1, 1) -> 24-bit PCM.
    With ``extra_chunk`` an odd-sized 'LIST' chunk precedes 'data' (padding
    byte included), as many editors write."""
    x = np.asarray(x, dtype=np.float64)
    if x.ndim == 1:
        x = x[:, None]
    n, ch = x.shape
    q = np.clip(np.round(x * 8388608.0), -8388608, 8388607).astype(np.int32).reshape(-1)
    b = q.astype("<i4").view(np.uint8).reshape(-1, 4)[:, :3].tobytes()
    fmt = struct.pack("<HHIIHH", 1, ch, fs, fs * 3 * ch, 3 * ch, 24)
    chunks = b"fmt " + struct.pack("<I", len(fmt)) + fmt
    if extra_chunk:
        info = b"INFOISFT\x05\x00\x00\x00test\x00"
        chunks += b"LIST" + struct.pack("<I", len(info)) + info + (b"\x00" if len(info) & 1 else b"")
    chunks += b"data" + struct.pack("<I", len(b)) + b + (b"\x00" if len(b) & 1 else b"")
    with open(path, "wb") as fh:
        fh.write(b"RIFF" + struct.pack("<I", 4 + len(chunks)) + b"WAVE" + chunks)
