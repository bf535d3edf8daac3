#!/usr/bin/env python
"""Evaluate enhanced WAV files against references (mirrors
open_universe/bin/eval_metrics.py:57-191 for the metrics computable offline:
si-sdr, lsd, si-lsd; pesq-wb when the ``pesq`` package is installed).

    python -m open_universe_amd.bin.eval_metrics enhanced/ --ref clean/ [--result out.json]

Files are matched by stem (``<deg>/<name>.wav`` <-> ``<ref>/<name>.wav``); the
per-file results and the mean over files (``summary``) are written as JSON.
"""
import argparse
import json
import sys
from collections import defaultdict
from pathlib import Path

import numpy as np

from open_universe_amd.audio import load_audio
from open_universe_amd.metrics import METRICS, pesq_wb


def summarize(results, ignore_inf=True):
    """Mean of every metric over the files (eval_metrics.py:57-76)."""
    total, count = defaultdict(float), defaultdict(int)
    for res in results.values():
        for k, v in res.items():
            if isinstance(v, str):
                continue
            if ignore_inf or not np.isinf(v):
                total[k] += v
                count[k] += 1
    out = {k: total[k] / count[k] for k in total}
    out["number"] = len(results)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("deg", type=Path)
    ap.add_argument("--ref", type=Path, required=True)
    ap.add_argument("--result", type=Path, default=None)
    ap.add_argument("--pesq", action="store_true", help="also PESQ-wb (needs the pesq package)")
    a = ap.parse_args(argv)
    results = {}
    for deg_p in sorted(a.deg.rglob("*.wav")):
        ref_p = a.ref / f"{deg_p.stem}.wav"
        if not ref_p.exists():
            continue
        deg, fs = load_audio(deg_p)
        ref, fs_ref = load_audio(ref_p)
        if deg.shape[0] > 1 or ref.shape[0] > 1:
            raise ValueError("Expected mono data")
        if fs != fs_ref:
            raise ValueError("ref and deg should have same sampling freq.")
        n = min(deg.shape[-1], ref.shape[-1])
        r, d = ref[0, :n], deg[0, :n]
        res = {k: f(r, d, fs) for k, f in METRICS.items()}
        if a.pesq:
            res["pesq-wb"] = pesq_wb(r, d, fs)
        results[deg_p.stem] = res
    out = {"summary": summarize(results), "files": results}
    txt = json.dumps(out, indent=1)
    if a.result:
        a.result.write_text(txt + "\n")
    print(json.dumps(out["summary"]))
    return 0


if __name__ == "__main__":
    sys.exit(main())
