#!/usr/bin/env python
"""Per-op (per U-Net level) HBM traffic and time of the conv stack.

GPU step (run under rocprofv3 --pmc, one counter set per pass):

    python tools/level_pmc.py run --config c4 [--batch B] --out ops.json

records the config's enhance plan (one warm enhance: tuning, graph), times
every op with ou_program_profile (a serial eager replay, HIP events around
each op) and writes the per-op rows; its LAST GPU work is one more serial
eager replay, whose conv-stack dispatches the analysis maps onto the ops.

CPU step:

    python tools/level_pmc.py analyze ops.json FETCH_CSV WRITE_CSV [--out table.json]

takes the last dispatches of the conv-stack kernels (conv_kernel,
conv_rkernel, conv_pkernel, conv_wkernel, conv_rreduce, block_kernel) in
dispatch order -- an op with K slices (tile bits 12-13) dispatches twice, every
other op once -- and reports per op and per geometry: time, algorithmic bytes,
counter bytes (FETCH_SIZE x 2 + WRITE_SIZE, the gfx950 correction of
tools/pmc_summary.py), counter / algorithmic, and time over the op's own roof
time (max of algorithmic bytes / 8 TB/s and FLOPs / MFMA peak).
"""
import argparse
import collections
import csv
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

CONV_KERNELS = ("conv_kernel", "conv_rkernel", "conv_skernel", "conv_pkernel", "conv_wkernel", "conv_rreduce",
                "conv_fdkernel", "conv_fukernel", "block_kernel")
HBM = 8000.0e9
PEAK = {0: 157.3e12, 1: 2516.6e12 / 3, 2: 2516.6e12}


def n_dispatch(row):
    if row["kind_name"] == "conv":
        return 2 if (row["tile"] >> 12) & 3 else 1
    return 1


def run(a):
    import torch

    import bench
    from open_universe_amd import _lib as L

    C = bench.CONFIGS[a.config]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if C.get("conv_prec") and "OUHIP_CONV_PREC" not in os.environ:
        os.environ["OUHIP_CONV_PREC"] = C["conv_prec"]
    cfg, model = bench.build_model(dev, arch=C["arch"], damped=C.get("damped", False))
    fs = int(cfg["fs"])
    B = a.batch or C["batch"]
    T = int((a.seconds or C["seconds"]) * fs)
    import numpy as np

    from open_universe_amd.utils.synthetic import synth_audio

    mix = torch.from_numpy(np.stack([synth_audio(T, fs, j)[0] for j in range(B)])).to(dev)
    rng = torch.Generator(device=dev).manual_seed(1028282)
    ekw = {"n_steps": C["n_steps"]} if C["n_steps"] else {}
    with torch.no_grad():
        model.enhance(mix, rng=rng, **ekw)
        torch.cuda.synchronize()
        plan = next(iter(model._plans.values()))
        st = torch.cuda.current_stream(dev).cuda_stream
        ms = plan.prog.profile(st)
        kinds = plan.prog.op_kinds()
        rows = []
        for i, (t, k) in enumerate(zip(ms, kinds)):
            if k not in (L.OP_CONV, L.OP_BLOCK):
                continue
            info = dict(plan.prog.info[i])
            rows.append({"i": i, "kind_name": "conv" if k == L.OP_CONV else "block", "ms": t,
                         "flops": plan.prog.flops[i], "bytes": plan.prog.bytes[i], **info})
        prec = model._get_engine().conv_prec
        plan.prog.profile(st)   # the replay whose dispatches 'analyze' maps onto the rows
        torch.cuda.synchronize()
    with open(a.out, "w") as fh:
        json.dump({"config": a.config, "batch": B, "T": T, "prec": prec, "rows": rows,
                   "gpu_ms_conv": sum(r["ms"] for r in rows)}, fh)
    print(f"level_pmc run: {len(rows)} conv-stack ops, {sum(r['ms'] for r in rows):.3f} ms", flush=True)


def short(name):
    import re

    name = name.strip().replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"<.*", "", name)
    return name.split("::")[-1].replace("void ", "").strip()


def read_counter(path, counter):
    per = collections.defaultdict(float)
    names = {}
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if row.get("Counter_Name") != counter:
                continue
            k = short(row["Kernel_Name"])
            if k not in CONV_KERNELS:
                continue
            d = int(row["Dispatch_Id"])
            per[d] += float(row["Counter_Value"])
            names[d] = k
    ids = sorted(per)
    return [(names[d], per[d]) for d in ids]


def label(r):
    if r["kind_name"] == "block":
        tag = "+down" if r.get("rate") else ("+in" if r.get("in") else ("+head" if r.get("head") else ""))
        return f"block C{r['C']}{tag} n{r['n']}"
    return f"conv m{r['m']} cin{r['cin']} fr{r['frame']} k{r['kt']} n{r['n']}" + (
        f" rout{r['rout']}" if r.get("rout") else "") + (f" fir{r['fir']}" if r.get("fir") else "")


def analyze(a):
    doc = json.load(open(a.ops))
    rows = doc["rows"]
    need = sum(n_dispatch(r) for r in rows)
    fetch = read_counter(a.fetch, "FETCH_SIZE")
    write = read_counter(a.write, "WRITE_SIZE")
    if len(fetch) < need or len(write) < need:
        raise SystemExit(f"{len(fetch)} / {len(write)} conv-stack dispatches in the counters, need {need}")
    fetch, write = fetch[-need:], write[-need:]
    j = 0
    peak = PEAK[doc.get("prec", 1)]
    for r in rows:
        n = n_dispatch(r)
        ks = [fetch[j + q][0] for q in range(n)]
        main = ks[0]
        want = "block_kernel" if r["kind_name"] == "block" else None
        if want and main != want or (not want and main == "block_kernel"):
            raise SystemExit(f"op {r['i']} ({label(r)}): dispatch {main} does not match")
        r["kernel"] = main
        r["pmc_bytes"] = sum(2.0 * 1024 * fetch[j + q][1] + 1024 * write[j + q][1] for q in range(n))
        r["roof_ms"] = 1e3 * max(r["bytes"] / HBM, r["flops"] / peak)
        j += n
    agg = collections.OrderedDict()
    for r in rows:
        k = label(r)
        g = agg.setdefault(k, {"geometry": k, "kernel": r["kernel"], "ops": 0, "ms": 0.0, "alg_bytes": 0.0,
                               "pmc_bytes": 0.0, "roof_ms": 0.0, "gflop": 0.0, "tile": r.get("tile")})
        g["ops"] += 1
        g["ms"] += r["ms"]
        g["alg_bytes"] += r["bytes"]
        g["pmc_bytes"] += r["pmc_bytes"]
        g["roof_ms"] += r["roof_ms"]
        g["gflop"] += r["flops"] / 1e9
    tab = []
    for g in agg.values():
        g["pmc_over_alg"] = round(g["pmc_bytes"] / max(g["alg_bytes"], 1.0), 3)
        g["frac_of_roof"] = round(g["roof_ms"] / max(g["ms"], 1e-9), 3)
        g["hbm_frac"] = round(g["alg_bytes"] / (g["ms"] * 1e-3) / HBM, 3) if g["ms"] else None
        g["ms"] = round(g["ms"], 4)
        g["roof_ms"] = round(g["roof_ms"], 4)
        g["alg_bytes"] = round(g["alg_bytes"])
        g["pmc_bytes"] = round(g["pmc_bytes"])
        g["gflop"] = round(g["gflop"], 3)
        tab.append(g)
    tab.sort(key=lambda g: -(g["ms"] - g["roof_ms"]))
    tot = {k: sum(r[k] for r in rows) for k in ("ms", "bytes", "pmc_bytes", "roof_ms", "flops")}
    out = {"config": doc["config"], "batch": doc["batch"], "T": doc["T"], "prec": doc.get("prec"),
           "ops": len(rows),
           "conv_ms": round(tot["ms"], 3), "roof_ms": round(tot["roof_ms"], 3),
           "frac_of_roof": round(tot["roof_ms"] / tot["ms"], 3),
           "alg_bytes": round(tot["bytes"]), "pmc_bytes": round(tot["pmc_bytes"]),
           "pmc_over_alg": round(tot["pmc_bytes"] / tot["bytes"], 3),
           "hbm_frac": round(tot["bytes"] / (tot["ms"] * 1e-3) / HBM, 3),
           "note": "ms: serial eager replay with HIP events per op (ou_program_profile); pmc: FETCH_SIZE x2 + "
                   "WRITE_SIZE of the same ops' dispatches; roof: max(alg bytes / 8 TB/s, FLOPs / MFMA peak); "
                   "rows sorted by time above roof",
           "by_geometry": tab}
    txt = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(txt + "\n")
    print(f"{out['config']} B={out['batch']}: conv {out['conv_ms']} ms, roof {out['roof_ms']} ms "
          f"({out['frac_of_roof']}), pmc/alg {out['pmc_over_alg']}, HBM frac {out['hbm_frac']}")
    print(f"{'geometry':44s} {'ops':>4s} {'ms':>9s} {'roof':>8s} {'frac':>6s} {'pmc/alg':>8s} kernel")
    for g in tab[: a.top]:
        print(f"{g['geometry']:44s} {g['ops']:4d} {g['ms']:9.3f} {g['roof_ms']:8.3f} {g['frac_of_roof']:6.3f} "
              f"{g['pmc_over_alg']:8.3f} {g['kernel']}")


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--config", default="c4")
    r.add_argument("--batch", type=int, default=None)
    r.add_argument("--seconds", type=float, default=None)
    r.add_argument("--out", required=True)
    z = sub.add_parser("analyze")
    z.add_argument("ops")
    z.add_argument("fetch")
    z.add_argument("write")
    z.add_argument("--out")
    z.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    run(a) if a.cmd == "run" else analyze(a)


if __name__ == "__main__":
    main()
