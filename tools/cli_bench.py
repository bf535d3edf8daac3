#!/usr/bin/env python
"""End-to-end CLI throughput over a folder of WAV files of distinct lengths
(VERDICT r1 item 6): N synthetic 16 kHz clips of 0.5-10 s, a PP16 checkpoint
with seeded synthetic weights, ``open_universe_amd.bin.enhance`` run in
process.  Reports audio seconds / wall seconds for the whole run (model load,
plan recording, tuning, file I/O included) and for the second pass over the
same folder (warm process), and the device memory high-water mark of each.

    python tools/cli_bench.py [--files 50] [--streams 2]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch
import yaml

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from open_universe_amd.configs import get_config  # noqa: E402
from open_universe_amd.networks.universe import UniverseGAN  # noqa: E402
from open_universe_amd.utils.synthetic import synth_audio, synth_state_dict  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=50)
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--profile", action="store_true", help="cProfile the second (warm) pass")
    a = ap.parse_args()
    from scipy.io import wavfile

    from open_universe_amd.bin import enhance as cli

    tmp = tempfile.mkdtemp(prefix="ou_cli_")
    cfg = get_config("pp16", None)
    m = UniverseGAN(**{k: v for k, v in cfg.items() if k != "_target_"})
    sd = m.state_dict()
    sd.update(synth_state_dict([(k, v.shape) for k, v in sd.items()], 0))
    os.makedirs(os.path.join(tmp, "exp"))
    ckpt = os.path.join(tmp, "exp", "weights.ckpt")
    torch.save({"state_dict": sd}, ckpt)
    with open(os.path.join(tmp, "exp", "config.yaml"), "w") as fh:
        yaml.safe_dump({"model": cfg}, fh)
    rng = np.random.default_rng(7)
    lengths = sorted(set(int(x) for x in rng.uniform(0.5, 10.0, size=a.files) * 16000))
    noisy = os.path.join(tmp, "noisy")
    os.makedirs(noisy)
    for i, n in enumerate(lengths):
        x = synth_audio(n, 16000, i)[0]
        wavfile.write(os.path.join(noisy, f"clip{i:03d}.wav"), 16000, (np.clip(x, -1, 1) * 32767).astype(np.int16))
    audio_s = sum(lengths) / 16000.0
    rows = []
    for rep in range(2):
        torch.cuda.reset_peak_memory_stats()
        t0 = time.perf_counter()
        argv = [noisy, os.path.join(tmp, f"out{rep}"), "--model", ckpt, "--streams", str(a.streams)]
        if a.profile and rep == 1:
            import cProfile
            import pstats

            cProfile.runctx("cli.main(argv)", globals(), {"cli": cli, "argv": argv}, "/tmp/cli.prof")
            pstats.Stats("/tmp/cli.prof", stream=sys.stderr).sort_stats("tottime").print_stats(25)
        else:
            cli.main(argv)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        rows.append({"pass": rep, "files": len(lengths), "audio_s": round(audio_s, 2), "wall_s": round(dt, 3),
                     "xrt": round(audio_s / dt, 1), "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2**30, 2)})
        print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
