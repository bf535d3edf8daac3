#!/usr/bin/env python
"""Folded vs FIR-applied anti-aliased rate-change convs, per layer geometry.

    python tools/fir_bench.py [--config c4|c2|c5] [--prec 1|2] [--only NAME]

For every score-network rate-change conv of the config (the shapes its plan
records: B items, level lengths of the config's clip), the tuner times every
tile of the folded form (3-frame weights, the other kernels) and of the
FIR-applied form (tile bit 17); prints ms per launch, the reference's
algorithmic TF/s and GB/s (engine.conv_desc's _flops / _bytes) and the ratio.
Random weights and inputs (timing does not depend on values).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from open_universe_amd import engine as E

# config: (batch, samples per item, channels, rates)
CONFIGS = {
    "c2": (1, 128000, 32, [2, 4, 4, 5]),
    "c5": (1, 960000, 32, [2, 4, 4, 5]),
    "c4": (32, 240240, 48, [2, 3, 5, 8]),
}


def layers(cfg):
    B, T, C, rates = CONFIGS[cfg]
    out, t = [], T
    for i, r in enumerate(rates):
        c = C * 2 ** i
        out.append((f"down{i}_r{r}", "down", c, 2 * c, r, t, B))
        out.append((f"up{i}_r{r}", "up", 2 * c, c, r, -(-t // r), B))
        t = -(-t // r)
    # the conditioner's st_convs (condition.py:53-59): level i -> the bottleneck,
    # kernel = stride = the product of the rates below level i (fir mode 3)
    t, top = T, C * 2 ** len(rates)
    for i in range(len(rates) - 1):
        rt = 1
        for r in rates[i:]:
            rt *= r
        out.append((f"st{i}_r{rt}", "st", C * 2 ** i, top, rt, t, B))
        t = -(-t // rates[i])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--prec", type=int, default=1)
    ap.add_argument("--only", default=None)
    ap.add_argument("--folded", type=int, default=1, help="0: skip tuning the folded form (slow at C4 sizes)")
    ap.add_argument("--tile", type=lambda v: int(v, 0), default=None,
                    help="with --only: run the FIR form on this tile --reps times, no tuning (PMC passes)")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = "cuda:0"
    E.enable_autotune(True)
    tuner = E.L.TUNER
    tot_f = tot_p = 0.0
    for name, direction, cin, cout, r, T, B in layers(a.config):
        if a.only and a.only != name:
            continue
        g = torch.Generator().manual_seed(0)
        shape = (cin, cout, r) if direction == "up" else (cout, cin, r)
        sd = {"p.conv.weight": torch.randn(shape, generator=g) * 0.1, "p.prelu.weight": torch.tensor([0.25]),
              "p.bias": torch.randn(cout, generator=g)}
        spec = (E.spec_down(sd, "p", r, direction == "down") if direction in ("down", "st")
                else E.spec_up(sd, "p", r, True))
        cw = E.make_conv(spec, dev, prec=a.prec)
        x = E.Act(torch.randn(B, cin, T, device=dev))
        if direction != "up":
            y = E.new_act(B, cout, -(-T // r), dev)
            d = E.conv_desc(cw, x, y)
        else:
            y = E.new_act(B, cout, r * T, dev)
            d = E.conv_desc(cw, x, y, n_frames=T, valid_len=r * T, res1=y, s1=float(E.NF2))
        if a.tile is not None:   # a fixed FIR tile, launched --reps times (counter passes)
            f = E.fir_desc(d)
            f.tile = a.tile
            lib = E.L.load()
            st = torch.cuda.current_stream().cuda_stream
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            E.L.run_now(E.L.OP_CONV, f, st)
            e0.record()
            for _ in range(a.reps):
                E.L.run_now(E.L.OP_CONV, f, st)
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1) / a.reps
            print(f"{name:12s} FIR tile 0x{a.tile:x}: {ms * 1e3:9.1f} us, {d._flops / 1e9 / ms:6.1f} TF/s, "
                  f"{d._bytes / 1e9 / ms:6.2f} TB/s")
            continue
        tp, ms_p = tuner.pick(d) if a.folded else (-1, float("nan"))
        if cw.fir is None:
            print(f"{name:12s} folded {ms_p * 1e3:9.1f} us  (no FIR form)")
            continue
        f = E.fir_desc(d)
        tf, ms_f = tuner.pick(f)
        tot_f += ms_f
        tot_p += ms_p
        gf = d._flops / 1e9
        gb = d._bytes / 1e9
        print(f"{name:12s} B {B:2d} T {T:7d} cin {cin:4d} cout {cout:4d}: folded {ms_p * 1e3:9.1f} us "
              f"(tile 0x{tp:x}, {gf / ms_p:6.1f} TF/s)  FIR {ms_f * 1e3:9.1f} us (tile 0x{tf:x}, "
              f"{gf / ms_f:6.1f} TF/s, {gb / ms_f:6.2f} TB/s)  x{ms_p / ms_f:5.2f}", flush=True)
    print(f"total: folded {tot_p:.3f} ms  FIR {tot_f:.3f} ms per pass (x{tot_p / max(tot_f, 1e-9):.2f})")


if __name__ == "__main__":
    main()
