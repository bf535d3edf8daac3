#!/usr/bin/env python
"""Enhance a WAV / FLAC file or a folder of them (mirrors the reference's
open_universe/bin/enhance.py:1-192): same positional arguments, ``--model``,
``--model-strict``, ``--seed``, ``--device`` and the ``enhance()`` options
added from the model's signature (``inference_utils.add_enhance_arguments``).
The folder structure is kept.

Differences: audio is resampled to ``model.fs`` and back on the GPU
(``audio.resample``); WAV and FLAC are read (FLAC by the native decoder,
``audio.load_flac``), mp3 is not; the model must be a local checkpoint
(the Hugging Face hub needs the network).  Files are enhanced in groups of
``--chunk`` with ``--streams`` clips in flight (Universe.enhance_many).  Under
torchrun (WORLD_SIZE > 1) each rank enhances its share of the files on
``cuda:LOCAL_RANK`` (``sharding.shard_utterances``, balanced by file size) --
no collectives.

Noise: as in the reference (bin/enhance.py:71-73,147-148,173-189), one
generator seeded with ``--seed`` draws every file's noise in the order
``rglob`` lists the files (suffix matched case-sensitively).  A rank draws and
discards the noise of the files other ranks enhance (``Universe.skip_noise``,
from the file headers), so every file gets the same noise -- and the same
output -- whatever the world size.

    python -m open_universe_amd.bin.enhance noisy/ enhanced/ --model exp/ckpt.ckpt
    python -m torch.distributed.run --nproc-per-node 8 -m open_universe_amd.bin.enhance noisy/ out/ --model ...
"""
import argparse
import os
import sys
from pathlib import Path

import torch

from open_universe_amd import inference_utils
from open_universe_amd.audio import audio_info, load_audio, resample, resampled_len, save_audio
from open_universe_amd.sharding import dist_env, shard_utterances

AUDIO_SUFFIXES = [".wav", ".flac"]


def find_files(path):
    """(files, root, is_dir) as bin/enhance.py:46-58: rglob order, suffix
    matched case-sensitively (the order fixes which noise each file gets)."""
    if not path.is_dir():
        return [path], path.parent, False
    return [p for p in path.rglob("*") if p.suffix in AUDIO_SUFFIXES], path, True


def main(argv=None):
    parser = argparse.ArgumentParser(description="Enhance a file or a directory of audio files")
    parser.add_argument("input", type=Path, help="Path to an audio file or a folder of audio files")
    parser.add_argument("output", type=Path, help="Output path; for a folder the structure is retained")
    parser.add_argument("--model", type=str, required=True, help="Local checkpoint (.ckpt) of the model")
    parser.add_argument("--model-strict", action="store_true", help="Strict state-dict loading")
    parser.add_argument("--seed", type=int, default=1028282, help="Seed of the sampler noise")
    parser.add_argument("--device", type=str, default=None, help="cuda:X (default: cuda:LOCAL_RANK)")
    parser.add_argument("--streams", type=int, default=2,
                        help="clips in flight at once on separate HIP streams (Universe.enhance_many); 1 = one "
                             "enhance() per file, as the reference")
    parser.add_argument("--chunk", type=int, default=8, help="files read, enhanced and written per group")
    args, _ = parser.parse_known_args(argv)

    rank, local, world = dist_env()
    device = args.device or f"cuda:{local}"
    if not device.startswith("cuda") or not torch.cuda.is_available():
        raise SystemExit("open_universe_amd runs on a ROCm device (cuda:X); the CPU path is the reference")
    torch.cuda.set_device(torch.device(device))
    model = inference_utils.load_model(args.model, device=device, strict=args.model_strict)
    rng = torch.Generator(device=device)
    rng.manual_seed(args.seed)

    inference_utils.add_enhance_arguments(model, parser)
    args = parser.parse_args(argv)
    groups = {g.title: {a.dest: getattr(args, a.dest, None) for a in g._group_actions}
              for g in parser._action_groups}
    enhance_kwargs = dict(groups.get("enhance", {}))
    enhance_kwargs["rng"] = rng

    all_files, root, is_dir = find_files(args.input)
    mine = list(range(len(all_files)))
    if world > 1:
        mine = shard_utterances([p.stat().st_size for p in all_files], world)[rank]
    files = [all_files[i] for i in mine]
    # the files before each of mine (in the global order) that other ranks
    # enhance: their noise is drawn and discarded right before mine
    skip_before, prev = [], -1
    for i in mine:
        skip_before.append(all_files[prev + 1:i])
        prev = i
    noise_kw = {k: enhance_kwargs.get(k) for k in ("n_steps", "target", "use_aux_signal", "ensemble",
                                                  "warm_start")}

    def skip(paths):
        for p in paths:
            ch, n, fs = audio_info(p)
            model.skip_noise((ch, resampled_len(n, fs, model.fs)), rng, **noise_kw)

    def out_path(path):
        if is_dir:
            return args.output / path.relative_to(root)
        if args.output.is_dir() or args.output.suffix == "":
            return args.output / path.name
        return args.output

    # enhance_many covers the sampler options below; any other option (ensemble,
    # aux signal, warm start, known-answer target) goes file by file
    many_ok = args.streams > 1 and all(
        enhance_kwargs.get(k) in (None, False) for k in ("target", "fake_score_snr", "use_aux_signal", "ensemble",
                                                         "warm_start"))
    many_kw = {k: enhance_kwargs.get(k) for k in ("n_steps", "epsilon", "keep_rms", "rng")}
    step = max(1, args.chunk) if many_ok else 1
    for i in range(0, len(files), step):
        group = files[i:i + step]
        loaded = [load_audio(p) for p in group]
        with torch.no_grad():
            xs = [resample(a.to(device), fs, model.fs) for a, fs in loaded]
            if many_ok:
                ys = model.enhance_many(xs, streams=args.streams, pre_noise=lambda j: skip(skip_before[i + j]),
                                        **many_kw)
            else:
                ys = []
                for j, x in enumerate(xs):
                    skip(skip_before[i + j])
                    ys.append(model.enhance(x, **enhance_kwargs))
            ys = [resample(y, model.fs, fs) for y, (_, fs) in zip(ys, loaded)]
        for path, y, (_, fs) in zip(group, ys, loaded):
            out = out_path(path)
            out.parent.mkdir(parents=True, exist_ok=True)
            save_audio(out, y, fs)
            print(f"[rank {rank}] {path} -> {out}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
