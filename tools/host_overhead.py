#!/usr/bin/env python
"""Host-side cost of one enhance() call at C2 (the GPU idles while it runs).

    python tools/host_overhead.py [--calls 30] [--profile]

Prints the wall time per call, the host time spent in each part of the call
(plan.submit = input copy + noise draws + graph launch, then the status check,
then the output copy), and with --profile the top cProfile entries."""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=30)
    ap.add_argument("--profile", action="store_true")
    a = ap.parse_args()
    import bench
    from open_universe_amd.utils.synthetic import synth_audio

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg, model = bench.build_model(dev, arch="pp16")
    fs = int(cfg["fs"])
    mix = torch.from_numpy(synth_audio(8 * fs, fs, 0)[0][None]).to(dev)
    rng = torch.Generator(device=dev).manual_seed(0)
    with torch.no_grad():
        for _ in range(3):
            model.enhance(mix, rng=rng)
        torch.cuda.synchronize()
        plan = next(iter(model._plans.values()))
        walls, sub, chk, cln = [], [], [], []
        for _ in range(a.calls):
            t0 = time.perf_counter()
            out = plan.submit(mix[:, None, :], rng)
            t1 = time.perf_counter()
            plan.check()
            t2 = time.perf_counter()
            out.clone()
            t3 = time.perf_counter()
            sub.append(t1 - t0), chk.append(t2 - t1), cln.append(t3 - t2)
        for _ in range(a.calls):
            t0 = time.perf_counter()
            model.enhance(mix, rng=rng)
            walls.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
        med = lambda v: 1e6 * float(np.median(v))
        print(f"enhance() wall {med(walls):.1f} us per call; plan.submit host {med(sub):.1f} us, "
              f"check (waits for the GPU) {med(chk):.1f} us, output clone {med(cln):.1f} us")
        if a.profile:
            pr = cProfile.Profile()
            pr.enable()
            for _ in range(a.calls):
                model.enhance(mix, rng=rng)
            pr.disable()
            pstats.Stats(pr).sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()
