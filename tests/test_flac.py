"""FLAC input decoding (csrc/ou_flac.cpp, host code: runs without a GPU).

The reference CLI reads .wav/.mp3/.flac through torchaudio.load
(open_universe/bin/enhance.py:33,61-64).  Neither torchaudio nor libFLAC is
in this image, so the streams are made by tests/flac_writer.py, an
independent encoder written from RFC 9639, covering every subframe type,
Rice form, stereo mode and header code the decoder handles.  FLAC is
lossless: the decoder must return the encoded integers exactly, scaled by
2^-(bps-1) as torchaudio.load scales integer PCM.  (No reference-produced
.flac file exists offline: parity against torchaudio is unpinned.)
"""
import numpy as np
import pytest

from open_universe_amd import _lib as L
from open_universe_amd import audio

import flac_writer as fw


def _signal(rng, ch, n, bps):
    t = np.arange(n)
    hi = (1 << (bps - 1)) - 1
    x = np.stack([0.6 * np.sin(2 * np.pi * (0.01 + 0.003 * c) * t) + 0.05 * rng.standard_normal(n)
                  for c in range(ch)])
    return np.clip(np.round(x * hi), -hi - 1, hi).astype(np.int64)


def _decode(tmp_path, data, name="x.flac"):
    p = tmp_path / name
    p.write_bytes(data)
    x, fs = audio.load_audio(p)
    return x.numpy(), fs


def _mono_frames(n):
    kinds = [{"kind": ("fixed", o)} for o in range(5)]
    kinds += [{"kind": "verbatim"},
              {"kind": "lpc", "lpc": ([3, -3, 1], 12, 0)},
              {"kind": "lpc", "lpc": ([1900, -950], 12, 10), "porder": 2},
              {"kind": ("fixed", 2), "porder": 3, "method": 1},
              {"kind": ("fixed", 1), "escape": True, "porder": 1}]
    return [{"n": n, "sub": [k]} for k in kinds]


def test_mono_every_subframe_type(tmp_path):
    rng = np.random.default_rng(0)
    frames = _mono_frames(512)
    x = _signal(rng, 1, 512 * len(frames), 16)
    data = fw.encode(x, 16000, 16, frames)
    y, fs = _decode(tmp_path, data)
    assert fs == 16000 and y.shape == x.shape
    np.testing.assert_array_equal(y, x.astype(np.float32) / 32768.0)


def test_constant_and_wasted_bits(tmp_path):
    n = 256
    x = np.concatenate([np.full(n, -1234), (np.arange(n) % 7 - 3) * 16, np.zeros(n)])[None].astype(np.int64)
    frames = [{"n": n, "sub": [{"kind": "constant"}]},
              {"n": n, "sub": [{"kind": ("fixed", 1), "wasted": 4}]},
              {"n": n, "sub": [{"kind": "constant", "wasted": 0}]}]
    y, _ = _decode(tmp_path, fw.encode(x, 8000, 16, frames))
    np.testing.assert_array_equal(y, x.astype(np.float32) / 32768.0)


@pytest.mark.parametrize("mode", [0, 8, 9, 10])
@pytest.mark.parametrize("bps", [16, 24])
def test_stereo_decorrelation_modes(tmp_path, mode, bps):
    rng = np.random.default_rng(mode + bps)
    n = 1152
    x = _signal(rng, 2, 3 * n, bps)
    sub = [{"kind": ("fixed", 2), "porder": 2}, {"kind": "lpc", "lpc": ([2, -1], 4, 0)}]
    frames = [{"n": n, "mode": mode, "sub": sub} for _ in range(3)]
    y, fs = _decode(tmp_path, fw.encode(x, 48000, bps, frames))
    assert fs == 48000
    np.testing.assert_array_equal(y, x.astype(np.float32) / float(1 << (bps - 1)))


@pytest.mark.parametrize("bps", [8, 12, 20])
def test_block_size_and_sample_size_codes(tmp_path, bps):
    """Explicit 8- and 16-bit block sizes (a short last block), sample size
    taken from the frame header and from STREAMINFO, total left 0 in
    STREAMINFO (the decoder counts the frames)."""
    rng = np.random.default_rng(bps)
    frames = [{"n": 4096, "sub": [{"kind": ("fixed", 3)}]},
              {"n": 1000, "bs_code": 7, "sub": [{"kind": ("fixed", 2)}], "ss_from_streaminfo": True},
              {"n": 100, "bs_code": 6, "sub": [{"kind": "verbatim"}]}]
    x = _signal(rng, 1, 5196, bps)
    y, fs = _decode(tmp_path, fw.encode(x, 24000, bps, frames, total_in_streaminfo=False))
    assert fs == 24000
    np.testing.assert_array_equal(y, x.astype(np.float32) / float(1 << (bps - 1)))


@pytest.mark.parametrize("mode", [8, 9, 10])
def test_32_bit_stereo_side_channel_needs_33_bits(tmp_path, mode):
    """RFC 9639: the side channel of a 32-bit stream is a 33-bit signal;
    channels at opposite full scale make it use the 33rd bit."""
    n = 256
    lo, hi = -(1 << 31), (1 << 31) - 1
    left = np.where(np.arange(n) % 2 == 0, hi, lo).astype(np.int64)
    # frame 2: near opposite full scale but smooth, so a FIXED predictor's
    # residuals stay small (RFC 9639 keeps residuals within 32 bits) while
    # its 33-bit warm-up sample and predictions do not
    ramp = hi - (np.arange(n) % 64) * 1000
    x = np.concatenate([np.stack([left, -left - 1]), np.stack([ramp, -ramp - 1])], axis=1)
    frames = [{"n": n, "mode": mode, "sub": [{"kind": "verbatim"}] * 2},
              {"n": n, "mode": mode, "sub": [{"kind": ("fixed", 1)}] * 2}]
    y, _ = _decode(tmp_path, fw.encode(x, 48000, 32, frames))
    np.testing.assert_array_equal(y, x.astype(np.float32) / float(1 << 31))


@pytest.mark.parametrize("tail", [b"TAG" + bytes(125), bytes(64)])
def test_trailing_bytes_after_last_frame(tmp_path, tail):
    """An ID3v1 tag or padding after the last frame is ignored once every
    sample STREAMINFO announced is decoded (as libFLAC does); the same bytes
    before the end of the samples are still a lost frame sync."""
    rng = np.random.default_rng(3)
    frames = _mono_frames(256)[:3]
    x = _signal(rng, 1, 768, 16)
    data = fw.encode(x, 16000, 16, frames)
    y, _ = _decode(tmp_path, data + tail)
    np.testing.assert_array_equal(y, x.astype(np.float32) / 32768.0)
    if tail[:3] != b"TAG":   # padding where a frame should start
        cut = data[: len(data) - 10]
        with pytest.raises(L.OuHipError, match="flac"):
            _decode(tmp_path, cut + tail)


def test_damaged_stream_fails_loudly(tmp_path):
    rng = np.random.default_rng(1)
    frames = _mono_frames(256)[:3]
    x = _signal(rng, 1, 768, 16)
    data = bytearray(fw.encode(x, 16000, 16, frames))
    data[-40] ^= 0x10   # a residual bit of the last frame
    with pytest.raises(L.OuHipError, match="flac"):
        _decode(tmp_path, bytes(data))
    with pytest.raises(L.OuHipError, match="fLaC"):
        _decode(tmp_path, b"RIFF" + bytes(40))


def test_cli_lists_flac_inputs(tmp_path):
    from open_universe_amd.bin import enhance as cli

    assert ".flac" in cli.AUDIO_SUFFIXES


@pytest.mark.parametrize("ch,n,bits", [(1, 1, 16), (1, 4096, 24), (2, 10000, 16), (2, 12345, 24)])
def test_encoder_round_trip(tmp_path, ch, n, bits):
    """ou_flac_encode (the CLI's .flac output) -> ou_flac_decode: the PCM the
    encoder quantised comes back exactly (block sizes from the table and
    explicit 16-bit ones; FIXED-2 and VERBATIM subframes)."""
    import torch

    rng = np.random.default_rng(n)
    t = np.arange(n)
    x = np.stack([0.5 * np.sin(2 * np.pi * 0.013 * (c + 1) * t) for c in range(ch)])
    if n > 100:
        x[:, 50:100] = rng.uniform(-1.2, 1.2, (ch, 50))   # noise burst + clipping: VERBATIM blocks
    x = x.astype(np.float32)
    p = tmp_path / "o.flac"
    audio.save_audio(p, torch.from_numpy(x), 22050)
    y, fs = audio.load_audio(p)
    full = float(1 << (bits - 1)) if bits == 24 else None
    q = np.clip(np.rint(x.astype(np.float64) * (1 << (bits - 1))), -(1 << (bits - 1)), (1 << (bits - 1)) - 1)
    if bits == 24:   # save_audio writes 24-bit
        assert fs == 22050 and y.shape == (ch, n)
        np.testing.assert_array_equal(y.numpy(), (q / full).astype(np.float32))
    else:
        from open_universe_amd import _lib as LL
        import ctypes

        lib = LL.load()
        a = np.ascontiguousarray(x)
        cap = lib.ou_flac_encode_bound(ch, n, 16)
        buf = (ctypes.c_uint8 * cap)()
        got = lib.ou_flac_encode(a.ctypes.data, ch, n, 22050, 16, buf, cap)
        assert 0 < got <= cap
        y16, _ = _decode(tmp_path, bytes(buf)[:got], "o16.flac")
        np.testing.assert_array_equal(y16, (q / 32768.0).astype(np.float32))
