#!/usr/bin/env python
"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output (stdin)."""
import re
import sys

rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"remark:\s+(?:\S+:\d+:\d+:\s+)?(.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        nm = t.split(":", 1)[1].strip()
        a = re.search(r"kernelI(.*?)EEv", nm)
        base = re.search(r"N_\d+([A-Za-z_]+?kernel)I", nm)
        cur = {"n": (base.group(1) if base else nm[:30]) + "<" +
               ",".join(re.findall(r"Li(\d+)E", a.group(1) if a else "")) + ">"}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    print(f"{r['n']:40s} vgpr {r.get('VGPRs', '?'):>4} agpr {r.get('AGPRs', '?'):>4} "
          f"scratch {r.get('ScratchSize [bytes/lane]', '?'):>4} occ {r.get('Occupancy [waves/SIMD]', '?')}")
