#!/usr/bin/env python
"""Aggregate a rocprofv3 ``*_kernel_stats.csv`` by kernel family (template
instances of one kernel summed), so its per-launch average can be compared with
bench.py's HIP-event figure.

    python tools/kstats_summary.py KERNEL_STATS_CSV [--per N] [--out JSON]

``--per N`` divides calls and time by N (e.g. the number of enhance() calls in
the profiled run) to give per-enhance figures.
"""
import argparse
import collections
import csv
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import short  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--per", type=float, default=1.0)
    ap.add_argument("--out")
    a = ap.parse_args()
    agg = collections.defaultdict(lambda: [0, 0.0])
    with open(a.csv) as fh:
        for r in csv.DictReader(fh):
            k = short(r["Name"])
            agg[k][0] += int(r["Calls"])
            agg[k][1] += float(r["TotalDurationNs"])
    tot = sum(v[1] for v in agg.values())
    # runtime copy / fill kernels come from engine construction (weight
    # uploads, workspace zeroing) and input staging, not from the recorded
    # enhance() program: reported with their totals, not per enhance
    setup = {"__amd_rocclr_copyBuffer", "__amd_rocclr_fillBufferAligned", "__amd_rocclr_copyBufferAligned"}
    rows = {}
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        row = {"calls": v[0], "total_ms": round(v[1] / 1e6, 3), "avg_us": round(v[1] / v[0] / 1e3, 3),
               "pct": round(100 * v[1] / tot, 2)}
        if k in setup:
            row["note"] = "runtime copy/fill: engine setup and host->device staging, not part of enhance()"
        else:
            row.update(calls_per_enhance=round(v[0] / a.per, 2), ms_per_enhance=round(v[1] / 1e6 / a.per, 4))
        rows[k] = row
    txt = json.dumps({"source": a.csv, "per": a.per, "kernels": rows}, indent=1)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
