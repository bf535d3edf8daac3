"""Summarise a bench --dump-ops file per layer geometry."""
import collections
import json
import sys

rows = json.load(open(sys.argv[1]))
agg = collections.defaultdict(lambda: [0, 0.0, 0.0, None])
other = collections.defaultdict(float)
for r in rows:
    if r["kind"] != 1:
        other[r["kind"]] += r["ms"]
        continue
    key = (r["m"], r["cin"], r["frame"], r["kt"], r["n"], r["rout"])
    a = agg[key]
    a[0] += 1
    a[1] += r["ms"]
    a[2] += r["gflop"]
    a[3] = r["tile"]
tot = sum(v[1] for v in agg.values())
print("conv ms %.3f  other by kind %s" % (tot, {k: round(v, 3) for k, v in other.items()}))
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[: int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(k, "x%d" % v[0], "ms %.3f" % v[1], "TF/s %.1f" % (v[2] / max(v[1], 1e-9)), "tile", v[3])
