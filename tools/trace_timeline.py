#!/usr/bin/env python
"""Timeline of the last enhance in a rocprofv3 ``*_kernel_trace.csv``: the
GRU launches (their durations and the gaps between them -- the conv work on
the critical path) and, between GRU launches, how much conv time ran on each
hardware queue.

    python tools/trace_timeline.py KERNEL_TRACE_CSV --gru-per-enhance N
"""
import argparse
import csv
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import short  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--gru-per-enhance", type=int, required=True)
    a = ap.parse_args()
    rows = []
    with open(a.csv) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                         r.get("Queue_Id", "?")))
    rows.sort()
    gru = [i for i, r in enumerate(rows) if r[2] == "gru_ks_kernel"]
    k = a.gru_per_enhance
    if len(gru) < 2 * k:
        sys.exit("need two enhances of GRU launches")
    i0, i1 = gru[-2 * k], gru[-k]
    win = rows[i0:i1]
    t0 = win[0][0]
    print(f"window {len(win)} dispatches, wall {(win[-1][1] - t0) / 1e3:.1f} us")
    prev_end = None
    for i, (s, e, n, q) in enumerate(win):
        if n != "gru_ks_kernel":
            continue
        # conv kernels between the previous GRU's end and this one's start
        lo = prev_end if prev_end is not None else s
        busy = {}
        for s2, e2, n2, q2 in win:
            if n2 != "gru_ks_kernel" and s2 < s and e2 > lo:
                busy[q2] = busy.get(q2, 0) + min(e2, s) - max(s2, lo)
        during = {}
        for s2, e2, n2, q2 in win:
            if n2 != "gru_ks_kernel" and s2 < e and e2 > s:
                during[q2] = during.get(q2, 0) + min(e2, e) - max(s2, s)
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        print(f"GRU @{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:7.1f}  gap before {gap:7.1f}  "
              f"convs in gap (us/queue) {dict((q2, round(v / 1e3, 1)) for q2, v in busy.items())}  "
              f"convs during {dict((q2, round(v / 1e3, 1)) for q2, v in during.items())}")
        prev_end = e


if __name__ == "__main__":
    main()
