#!/usr/bin/env python
"""Compare per-layer conv time between two bench --dump-ops files."""
import collections
import json
import sys


def load(p):
    g = collections.defaultdict(lambda: [0, 0.0, 0.0, None])
    for x in json.load(open(p)):
        if x["kind"] != 1:
            continue
        k = (x["m"], x["cin"], x["frame"], x["kt"], x["n"], x["b"], x["rout"])
        g[k][0] += 1
        g[k][1] += x["ms"]
        g[k][2] += x["gflop"]
        g[k][3] = x["tile"]
    return g


a, b = load(sys.argv[1]), load(sys.argv[2])
print("m cin frame kt n b rout | cnt  msA  msB  TF/sA TF/sB tileA tileB")
for k in sorted(a, key=lambda k: -a[k][1]):
    va, vb = a[k], b.get(k, [0, 0, 0, None])
    tfa = va[2] / va[1] if va[1] else 0
    tfb = vb[2] / vb[1] if vb[1] else 0
    print(k, va[0], f"{va[1]:.3f} {vb[1]:.3f}  {tfa:5.1f} {tfb:5.1f}  {va[3]} {vb[3]}")
print(f"total {sum(v[1] for v in a.values()):.3f} {sum(v[1] for v in b.values()):.3f}")
