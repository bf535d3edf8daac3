"""CPU: WAV header parsing for the CLI's sharding pass (audio.audio_info, the
torchaudio.info fields bin/enhance.py reads: channels, frames, rate) against
what load_audio decodes, for every PCM container width including 24-bit."""
import numpy as np
import pytest
from scipy.io import wavfile

from open_universe_amd.audio import audio_info, load_audio
from wav_writer import write_wav24


@pytest.mark.parametrize("dtype", [np.int16, np.int32, np.uint8, np.float32, np.float64])
@pytest.mark.parametrize("ch", [1, 2])
def test_audio_info_matches_load_audio(tmp_path, dtype, ch):
    rng = np.random.default_rng(1)
    n = 1237
    x = rng.standard_normal((n, ch)) * 0.1
    if np.issubdtype(dtype, np.integer):
        info = np.iinfo(dtype)
        x = np.clip(x * info.max, info.min, info.max).astype(dtype)
    else:
        x = x.astype(dtype)
    p = tmp_path / "a.wav"
    wavfile.write(p, 22050, x if ch > 1 else x[:, 0])
    y, fs = load_audio(p)
    assert audio_info(p) == (ch, n, 22050) == (y.shape[0], y.shape[1], fs)


@pytest.mark.parametrize("ch,n", [(1, 1000), (2, 777), (1, 1)])
def test_audio_info_24bit(tmp_path, ch, n):
    """24-bit PCM (3-byte container): scipy's mmap reader refuses it; the
    header parser and load_audio both read it (odd-sized chunks padded)."""
    rng = np.random.default_rng(2)
    x = rng.uniform(-0.5, 0.5, (n, ch))
    p = tmp_path / "b.wav"
    write_wav24(p, 16000, x)
    assert audio_info(p) == (ch, n, 16000)
    y, fs = load_audio(p)
    assert fs == 16000 and y.shape == (ch, n)
    np.testing.assert_allclose(y.numpy().T, x, atol=1.0 / 8388608 + 1e-7)


def test_audio_info_rejects_non_wave(tmp_path):
    p = tmp_path / "c.wav"
    p.write_bytes(b"not a riff file at all")
    with pytest.raises(ValueError):
        audio_info(p)
