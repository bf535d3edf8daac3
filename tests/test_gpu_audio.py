"""F3 on the GPU: ``ou_resample`` (csrc/ou_audio.hip) against the oracle's
restatement of torchaudio.functional.resample (oracle/ou_oracle.py resample),
and the enhance CLI end to end (bin/enhance.py of the reference: resample to
model.fs, enhance, resample back, write).  Tolerance: fp32 with a different
summation order than conv1d -> max abs error <= 2e-6 * max|x| per output."""
import math

import numpy as np
import pytest
import torch

from open_universe_amd import _lib as L
from open_universe_amd.audio import load_audio, resample, save_audio
from oracle import ou_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("orig,new", [(48000, 16000), (16000, 24000), (44100, 16000), (22050, 16000),
                                      (8000, 16000), (16000, 48000), (24000, 16000), (1, 2), (2, 1)])
@pytest.mark.parametrize("n", [1, 7, 160, 16001, 96000])
def test_resample_matches_oracle(orig, new, n):
    g = torch.Generator().manual_seed(n + orig)
    x = torch.randn(3, n, generator=g)
    want = O.resample(x, orig, new)
    got = resample(x.to(DEV), orig, new)
    torch.cuda.synchronize()
    gcd = math.gcd(orig, new)
    assert got.shape == want.shape == (3, math.ceil(new // gcd * n / (orig // gcd)))
    err = (got.cpu() - want).abs().max().item()
    assert err <= 2e-6 * max(1.0, x.abs().max().item()), err


def test_resample_shapes_and_errors():
    x = torch.randn(2, 1, 3200, device=DEV)
    y = resample(x, 16000, 8000)
    assert y.shape == (2, 1, 1600)
    assert resample(x, 16000, 16000) is x
    with pytest.raises(L.OuHipError):
        resample(x.cpu(), 16000, 8000)
    # invalid table geometry is rejected by the C ABI, not run
    k = torch.zeros(2, 5, device=DEV)
    y = torch.empty(1, 10, device=DEV)
    rc = L.load().ou_resample(x.data_ptr(), 3200, y.data_ptr(), 10, 1, 3200, 10, k.data_ptr(), 2, 5, 1, 1,
                              torch.cuda.current_stream().cuda_stream)
    assert rc != 0


def test_enhance_cli_end_to_end(tmp_path):
    from scipy.io import wavfile

    from open_universe_amd.bin import enhance as cli
    from test_api_surface import _write_ckpt

    ckpt, _, _, _ = _write_ckpt(str(tmp_path), with_ema=False)
    src = tmp_path / "noisy"
    (src / "sub").mkdir(parents=True)
    rng = np.random.default_rng(0)
    wavfile.write(src / "a.wav", 48000, (rng.standard_normal(48000 // 2) * 3000).astype(np.int16))
    wavfile.write(src / "sub" / "b.wav", 16000, rng.standard_normal(12345).astype(np.float32) * 0.1)
    out = tmp_path / "enh"
    assert cli.main([str(src), str(out), "--model", ckpt, "--n_steps", "2", "--seed", "7"]) == 0
    for rel, fs, n in (("a.wav", 48000, 24000), ("sub/b.wav", 16000, 12345)):
        y, fs_out = load_audio(out / rel)
        assert fs_out == fs and y.shape[0] == 1
        assert abs(y.shape[-1] - n) <= 3, (rel, y.shape)     # 48k -> 16k -> 48k rounds up
        assert torch.isfinite(y).all() and y.abs().max() > 0
    # one generator per run, shared by the files in order (bin/enhance.py:146-147):
    # the same file and seed in a fresh run gives the same output
    outs = []
    for i in range(2):
        outs.append(tmp_path / f"enh{i}.wav")
        assert cli.main([str(src / "sub" / "b.wav"), str(outs[-1]), "--model", ckpt, "--n_steps", "2",
                         "--seed", "7"]) == 0
    a, _ = load_audio(outs[0])
    b, _ = load_audio(outs[1])
    assert torch.equal(a, b)


def test_enhance_cli_flac_in_flac_out(tmp_path):
    """A .flac input (decoded by ou_flac_decode) is enhanced and written back
    as .flac (ou_flac_encode), as the reference does through torchaudio."""
    import torch

    from open_universe_amd.bin import enhance as cli
    from test_api_surface import _write_ckpt

    ckpt, _, _, _ = _write_ckpt(str(tmp_path), with_ema=False)
    src = tmp_path / "noisy"
    src.mkdir()
    rng = np.random.default_rng(3)
    save_audio(src / "c.flac", torch.from_numpy((rng.standard_normal(20000) * 0.1).astype(np.float32)), 24000)
    x, fs = load_audio(src / "c.flac")
    assert fs == 24000 and x.shape == (1, 20000)
    out = tmp_path / "enh"
    assert cli.main([str(src), str(out), "--model", ckpt, "--n_steps", "2", "--seed", "7"]) == 0
    assert (out / "c.flac").read_bytes()[:4] == b"fLaC"
    y, fs_out = load_audio(out / "c.flac")
    assert fs_out == 24000 and y.shape[0] == 1 and abs(y.shape[-1] - 20000) <= 3
    assert torch.isfinite(y).all() and y.abs().max() > 0


@pytest.mark.parametrize("streams", [2, 1])
def test_enhance_cli_outputs_independent_of_world_size(tmp_path, monkeypatch, streams):
    """Every file's noise comes from the one --seed generator in the
    reference's file order (bin/enhance.py:71-73,147-148,173-189), whatever
    the world size: rank 0 and rank 1 of WORLD_SIZE=2 (both on cuda:0 here)
    together write outputs bit-identical to the single-rank run."""
    from scipy.io import wavfile

    from open_universe_amd.bin import enhance as cli
    from test_api_surface import _write_ckpt
    from wav_writer import write_wav24

    ckpt, _, _, _ = _write_ckpt(str(tmp_path), with_ema=False)
    src = tmp_path / "noisy"
    src.mkdir()
    rng = np.random.default_rng(5)
    lens = {"w0.wav": (16000, 9000), "w1.wav": (48000, 30000), "w2.wav": (16000, 4000), "w3.wav": (8000, 7000),
            "w4.wav": (16000, 12000)}
    for name, (fs, n) in lens.items():
        if name == "w3.wav":   # a 24-bit PCM file: audio_info parses its header on every rank
            write_wav24(src / name, fs, rng.standard_normal(n) * 0.1)
        else:
            wavfile.write(src / name, fs, (rng.standard_normal(n) * 0.1).astype(np.float32))
    common = ["--model", ckpt, "--n_steps", "3", "--seed", "11", "--device", "cuda:0", "--streams", str(streams),
              "--chunk", "2"]
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    assert cli.main([str(src), str(tmp_path / "one")] + common) == 0
    for r in (0, 1):
        monkeypatch.setenv("RANK", str(r))
        monkeypatch.setenv("LOCAL_RANK", "0")
        monkeypatch.setenv("WORLD_SIZE", "2")
        assert cli.main([str(src), str(tmp_path / "two")] + common) == 0
    for name in lens:
        a, _ = load_audio(tmp_path / "one" / name)
        b, _ = load_audio(tmp_path / "two" / name)
        assert torch.equal(a, b), name
