#!/usr/bin/env python
"""Per-kernel HBM traffic from rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_summary.py FETCH_CSV WRITE_CSV [--out JSON]

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  gfx950 correction
(MI355X_MICROARCH.md, HBM/rocprofv3 section): FETCH_SIZE reports half the bytes
of wide coalesced reads, so it is doubled; WRITE_SIZE is taken as is.  The
Infinity Cache (256 MiB) hits are counted as fetches too, so this is an upper
bound on HBM reads.
"""
import argparse
import collections
import csv
import json
import re


def short(name):
    name = name.strip().replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"<.*", "", name)
    return name.split("::")[-1].replace("void ", "").strip()


def lib_hash(path):
    import hashlib

    with open(path, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()[:16]


def read(path, counter):
    per = collections.defaultdict(float)  # (dispatch, kernel) -> value
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if row.get("Counter_Name") != counter:
                continue
            per[(row["Dispatch_Id"], short(row["Kernel_Name"]))] += float(row["Counter_Value"])
    agg = collections.defaultdict(lambda: [0, 0.0])
    for (_, k), v in per.items():
        agg[k][0] += 1
        agg[k][1] += v
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--out")
    ap.add_argument("--tag", default="")
    ap.add_argument("--enhances", type=int, default=None, help="enhance() calls in the profiled run")
    ap.add_argument("--config", default="c2", help="bench.py --config of the profiled run")
    ap.add_argument("--lib", default=None, help="the libouhip.so the profiled run loaded (its hash is recorded)")
    a = ap.parse_args()
    f, w = read(a.fetch, "FETCH_SIZE"), read(a.write, "WRITE_SIZE")
    rows = {}
    for k in sorted(set(f) | set(w)):
        n = max(f[k][0], w[k][0])
        fb = 2.0 * 1024.0 * f[k][1] / max(f[k][0], 1)
        wb = 1024.0 * w[k][1] / max(w[k][0], 1)
        rows[k] = {"dispatches": n, "fetch_bytes_per_launch": round(fb),
                   "write_bytes_per_launch": round(wb),
                   "traffic_bytes_per_launch": round(fb + wb)}
    out = {"tag": a.tag, "config": a.config, "correction": "FETCH_SIZE x2 (gfx950), KiB->bytes", "kernels": rows}
    # enhance() calls of the profiled run: one normalize_kernel each (a range
    # widening reruns the enhance, so the bench's step count alone undercounts)
    n_norm = max(f.get("normalize_kernel", [0])[0], w.get("normalize_kernel", [0])[0])
    if n_norm or a.enhances:
        out["enhances_profiled"] = n_norm or a.enhances
    if a.lib:
        # bench.py quotes these counters only for the same library build
        out["lib_sha16"] = lib_hash(a.lib)
    txt = json.dumps(out, indent=1)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
