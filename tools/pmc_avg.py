#!/usr/bin/env python
"""Average rocprofv3 counter values per dispatch of one kernel family.

    python tools/pmc_avg.py COUNTER_CSV [KERNEL_SUBSTRING]
"""
import collections
import csv
import sys

path = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "conv_kernel"
per = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(path)):
    if sub in r["Kernel_Name"]:
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
n = len(per)
keys = sorted({k for d in per.values() for k in d})
avg = {k: sum(d.get(k, 0.0) for d in per.values()) / max(n, 1) for k in keys}
print(f"{sub}: {n} dispatches")
for k in keys:
    print(f"  {k:28s} {avg[k]:16.1f}")
w = avg.get("SQ_WAVE_CYCLES")
if w:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if k in avg:
            print(f"  {k} / WAVE_CYCLES = {avg[k] / w:.3f}")
if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
    # MFMA busy is summed over all SIMDs (cycles); GUI_ACTIVE over 8 XCDs
    simds = 1024
    wall = avg["GRBM_GUI_ACTIVE"] / 8
    print(f"  MFMA busy fraction ~ {avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (simds * wall):.3f} (wall {wall:.0f} cyc)")
