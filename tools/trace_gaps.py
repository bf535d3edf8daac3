#!/usr/bin/env python
"""Busy time and idle gaps of the GPU in a rocprofv3 ``*_kernel_trace.csv``.

    python tools/trace_gaps.py KERNEL_TRACE_CSV [--last N]

Takes the last N dispatches of ``gru_ks_kernel`` as enhance() boundaries
(one enhance runs 10 GRU launches at PP16) and, over the window that spans
the last enhance, reports: wall time, the union of kernel-busy intervals (any
queue), the idle time between them, the number of idle gaps and their
distribution -- i.e. how much of an enhance is launch / dependency latency
rather than kernel time.
"""
import argparse
import csv
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import short  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--gru-per-enhance", type=int, default=10)
    a = ap.parse_args()
    rows = []
    with open(a.csv) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    gru = [i for i, r in enumerate(rows) if r[2] == "gru_ks_kernel"]
    k = a.gru_per_enhance
    if len(gru) < 2 * k:
        sys.exit("need at least two enhances of GRU launches in the trace")
    # window: from the first kernel after the previous enhance's last GRU's
    # decoder ... simplest robust choice: between the first GRU of the last
    # enhance and the first GRU of the one before, shifted to whole enhances
    i0, i1 = gru[-2 * k], gru[-k]
    win = rows[i0:i1]
    t0, t1 = win[0][0], win[-1][0]
    busy, gaps, cur_s, cur_e = 0, [], win[0][0], win[0][1]
    per_kernel = {}
    for s, e, n in win:
        per_kernel.setdefault(n, [0, 0])
        per_kernel[n][0] += 1
        per_kernel[n][1] += e - s
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    wall = t1 - t0
    gaps.sort()
    q = lambda p: gaps[min(len(gaps) - 1, int(p * len(gaps)))] / 1e3 if gaps else 0.0
    print(f"window: one enhance, {len(win)} dispatches, wall {wall / 1e6:.3f} ms")
    print(f"busy (union of kernels) {busy / 1e6:.3f} ms, idle {sum(gaps) / 1e6:.3f} ms in {len(gaps)} gaps; "
          f"gap us p10 {q(0.1):.2f} p50 {q(0.5):.2f} p90 {q(0.9):.2f} max {q(1.0):.2f}")
    for n, (c, t) in sorted(per_kernel.items(), key=lambda kv: -kv[1][1]):
        print(f"  {n:28s} x{c:4d} {t / 1e6:8.3f} ms")


if __name__ == "__main__":
    main()
