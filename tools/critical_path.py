#!/usr/bin/env python
"""Concurrent timeline of one enhance() plan by phase (GPU).

    python tools/critical_path.py [--config c2] [--reps 3] [--out JSON]

Records the config's plan (one warm enhance), then replays it eagerly with
the lanes on their own streams and a hipEvent before / after every op
(ou_program_trace), and reports per phase label (engine.py / plan.py set
them: "cond enc L2", "score dec L0", ...): the lane, first start, last end,
busy time; the diffusion-step boundaries (each score GRU's start and end);
the first step against a steady one.  Times are the median over --reps
replays.  Eager replay ran within 1 % of the graph replay in round 3
(profiles/bench_lanes_r03k.txt), so the schedule it shows is the graph's.
"""
import argparse
import collections
import json
import os
import statistics
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

KIND = {1: "conv", 2: "gru", 3: "embed", 4: "head", 5: "norm", 6: "invrms", 7: "rms", 8: "power", 9: "pad",
        10: "scale", 11: "finish", 12: "snake", 13: "memset", 14: "ens", 15: "block"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=None)
    ap.add_argument("--ops", action="store_true", help="print every op")
    a = ap.parse_args()
    import numpy as np
    import torch

    import bench
    from open_universe_amd import _lib as L
    from open_universe_amd.utils.synthetic import synth_audio

    C = bench.CONFIGS[a.config]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if C.get("conv_prec") and "OUHIP_CONV_PREC" not in os.environ:
        os.environ["OUHIP_CONV_PREC"] = C["conv_prec"]
    cfg, model = bench.build_model(dev, arch=C["arch"], damped=C.get("damped", False))
    fs = int(cfg["fs"])
    B = a.batch or C["batch"]
    T = int(C["seconds"] * fs)
    mix = torch.from_numpy(np.stack([synth_audio(T, fs, j)[0] for j in range(B)])).to(dev)
    rng = torch.Generator(device=dev).manual_seed(1028282)
    ekw = {"n_steps": C["n_steps"]} if C["n_steps"] else {}
    with torch.no_grad():
        for _ in range(2):
            model.enhance(mix, rng=rng, **ekw)
        torch.cuda.synchronize()
        plan = next(iter(model._plans.values()))
        st = torch.cuda.current_stream(dev).cuda_stream
        runs = [plan.prog.trace(st) for _ in range(a.reps)]
    prog = plan.prog
    kinds = prog.op_kinds()
    n = len(kinds)
    ops = []
    for i in range(n):
        if runs[0][i] is None:
            continue
        t0 = statistics.median(r[i][0] for r in runs)
        t1 = statistics.median(r[i][1] for r in runs)
        ops.append({"i": i, "kind": KIND.get(kinds[i], str(kinds[i])), "lane": prog.lanes[i],
                    "label": prog.labels[i], "t0": t0 * 1e3, "t1": t1 * 1e3, "info": prog.info[i]})
    wall = max(o["t1"] for o in ops)
    # diffusion steps: the score GRUs
    grus = [o for o in ops if o["kind"] == "gru" and o["label"] == "score gru"]
    phases = collections.OrderedDict()
    for o in ops:
        lab = o["label"]
        if lab.startswith("score") and lab != "score embed":
            # step index: score GRUs recorded up to this op (the encoder and
            # the GRU's input projection belong to the next GRU's step)
            k = sum(1 for g in grus if g["i"] <= o["i"])
            sidx = k if (lab.startswith("score dec") or o["kind"] == "gru") else k + 1
            lab = f"s{sidx} {lab[6:]}"
        ph = phases.setdefault(lab, {"label": lab, "lane": o["lane"], "ops": 0, "t0": o["t0"], "t1": o["t1"],
                                     "busy": 0.0})
        ph["ops"] += 1
        ph["t0"] = min(ph["t0"], o["t0"])
        ph["t1"] = max(ph["t1"], o["t1"])
        ph["busy"] += o["t1"] - o["t0"]
    lines = [f"{a.config} B={B}: wall {wall:.1f} us over {len(ops)} ops (eager lanes, median of {a.reps})"]
    lines.append(f"{'phase':22s} {'lane':>4s} {'ops':>4s} {'start':>8s} {'end':>8s} {'span':>7s} {'busy':>7s}")
    for ph in phases.values():
        lines.append(f"{ph['label']:22s} {ph['lane']:4d} {ph['ops']:4d} {ph['t0']:8.1f} {ph['t1']:8.1f} "
                     f"{ph['t1'] - ph['t0']:7.1f} {ph['busy']:7.1f}")
    lines.append("score GRUs (start, end, gap after the previous one's end):")
    prev = None
    for g in grus:
        lines.append(f"  {g['t0']:8.1f} {g['t1']:8.1f} dur {g['t1'] - g['t0']:6.1f}"
                     + (f" gap {g['t0'] - prev:7.1f}" if prev is not None else ""))
        prev = g["t1"]
    if len(grus) >= 3:
        steady = statistics.median(grus[k + 1]["t0"] - grus[k]["t0"] for k in range(1, len(grus) - 1))
        lines.append(f"first score GRU starts at {grus[0]['t0']:.1f} us, ends {grus[0]['t1']:.1f}; second starts "
                     f"{grus[1]['t0']:.1f}; steady step (GRU start to next GRU start) {steady:.1f} us")
        # step k runs from the start of "s{k} enc L0" to the start of the next one
        e = [phases[f"s{k} enc L0"]["t0"] for k in (1, 2, 3) if f"s{k} enc L0" in phases]
        if len(e) == 3:
            lines.append(f"first step: replay start -> s2 encoder start {e[1]:.1f} us "
                         f"(prep + conditioner + step 1; score step 1 alone {e[1] - e[0]:.1f} us); "
                         f"steady step (s2 -> s3 encoder start) {e[2] - e[1]:.1f} us; "
                         f"first-step excess {e[1] - (e[2] - e[1]):.1f} us")
    if a.ops:
        for o in ops:
            lines.append(f"{o['i']:4d} L{o['lane']} {o['t0']:8.1f} {o['t1']:8.1f} {o['t1'] - o['t0']:6.1f} "
                         f"{o['kind']:6s} {o['label']:14s} {json.dumps(o['info'])}")
    txt = "\n".join(lines)
    print(txt, flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump({"config": a.config, "batch": B, "wall_us": wall, "phases": list(phases.values()),
                       "ops": ops}, fh)


if __name__ == "__main__":
    main()
