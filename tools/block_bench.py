#!/usr/bin/env python
"""Microbenchmark: one fused ConvBlock (ou_block) against the three tuned
ou_conv launches it replaces, at the PP16 level geometries (B = 1, 8 s) or
PP24's at C4's clip (--family pp24 --batch 32).

    python tools/block_bench.py [--reps 50] [--levels 0,1,2,3] [--family pp24 --batch 32 --fused-only]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from open_universe_amd import _lib as L  # noqa: E402
from open_universe_amd import engine as E  # noqa: E402

DEV = "cuda:0"
LEVELS = [(32, 128160), (64, 64080), (128, 16020), (256, 4005), (512, 801)]
# PP24 at C4's clip (10.01 s at 24 kHz; run with --batch 32 for the bench's batch)
LEVELS24 = [(48, 240240), (96, 120120), (192, 40040), (384, 8008), (768, 1001)]


def specs(C, g):
    out = []
    for k in (5, 3, 3):
        w = torch.randn(C, C, k, generator=g) / np.sqrt(C * k)
        out.append(E.ConvSpec(w.numpy(), C, 1, (k - 1) // 2, 1, 0.25, (0.1 * torch.randn(C, generator=g)).numpy(),
                              ref_macs=float(w.numel())))
    return out


COPIES = 20   # the op is recorded this many times into one graph: one
              # hipGraphLaunch (~10-20 us of host time) per COPIES launches


def time_prog(prog, reps):
    """Device microseconds per recorded op sequence (prog holds COPIES of it)."""
    stream = torch.cuda.current_stream().cuda_stream
    prog.run(stream)
    torch.cuda.synchronize()
    prog.capture()
    prog.launch(stream)
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(max(1, reps // 10)):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        prog.launch(stream)
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / COPIES)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--levels", default="0,1,2,3")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--family", default="pp16", choices=["pp16", "pp24"])
    ap.add_argument("--fused-only", action="store_true", help="skip the three-launch form (counter passes)")
    ap.add_argument("--dbg", default="", help="comma list of ou_block diagnostic masks to time as well "
                                                "(1 no input loads, 2 no MFMA stages, 4 no output pass)")
    a = ap.parse_args()
    E.enable_autotune(True)
    status = torch.zeros(4, dtype=torch.int32, device=DEV)
    E._PREP_STATUS = status.data_ptr() + 4
    ks = torch.empty(E.KSWS_BYTES // 4, dtype=torch.float32, device=DEV)
    E._PREP_KSWS = (ks.data_ptr(), E.KSWS_BYTES)
    rows = []
    for li in [int(x) for x in a.levels.split(",")]:
        C, T = (LEVELS24 if a.family == "pp24" else LEVELS)[li]
        g = torch.Generator().manual_seed(li)
        sp = specs(C, g)
        cws = [E.make_conv(s, DEV, prec=1) for s in sp]
        fused = E.prep_fused(sp, C, 1, DEV)
        bw = E.BlockW(C, "none", None, *cws, None, fused)
        B = a.batch
        h = E.Act(torch.randn(B, C, T, device=DEV))
        out, tA, tB = (E.new_act(B, C, T, DEV) for _ in range(3))
        res = {}
        for fz in (True,) if a.fused_only else (True, False):
            if not fz:
                bw.fused = None
            prog = L.Program()
            for _ in range(COPIES):
                E.rec_block(prog, bw, h, out, tA, tB)
            res["fused_us" if fz else "unfused_us"] = round(time_prog(prog, a.reps), 2)
            bw.fused = fused
        for mask in [int(x) for x in a.dbg.split(",") if x]:
            orig = E.block_desc

            def patched(*args, **kw):
                dd = orig(*args, **kw)
                dd.dbg = mask
                return dd

            E.block_desc = patched
            try:
                prog = L.Program()
                for _ in range(COPIES):
                    E.rec_block(prog, bw, h, out, tA, tB)
                res[f"dbg{mask}_us"] = round(time_prog(prog, a.reps), 2)
            finally:
                E.block_desc = orig
        flops = 2.0 * B * T * C * C * 11
        rows.append({"C": C, "T": T, "B": B, **res, "frames_per_wg": L.load().ou_block_frames(C),
                     "tflops_fused": round(flops / res["fused_us"] / 1e6, 1)})
        print(json.dumps(rows[-1]), flush=True)
    assert int(status.abs().sum()) == 0


if __name__ == "__main__":
    main()
