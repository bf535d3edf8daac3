#!/usr/bin/env bash
# PMC pass over tools/block_bench.py (fused ConvBlock kernel): wave-state and
# instruction-mix counters, one rocprofv3 run per counter set.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$ROOT/gpurun_out"
mkdir -p "$O"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d "$O/bpmc1" -o pmc -- \
    python3 "$ROOT/tools/block_bench.py" --levels "${LEVELS:-0,1,2}" --reps 10 > "$O/bpmc1.out" 2> "$O/bpmc1.err" &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU --output-format csv -d "$O/bpmc2" -o pmc -- \
    python3 "$ROOT/tools/block_bench.py" --levels "${LEVELS:-0,1,2}" --reps 10 > "$O/bpmc2.out" 2> "$O/bpmc2.err" &&
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE --output-format csv -d "$O/bpmc3" -o pmc -- \
    python3 "$ROOT/tools/block_bench.py" --levels "${LEVELS:-0,1,2}" --reps 10 > "$O/bpmc3.out" 2> "$O/bpmc3.err"
rc=$?
cd "$ROOT"
python3 - "$O" <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
for tag in ("bpmc1", "bpmc2", "bpmc3"):
    f = glob.glob(f"{O}/{tag}/**/*counter_collection.csv", recursive=True)
    if not f:
        print(tag, "no csv"); continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"]
        if "block_kernel" not in k: continue
        key = k.split("block_kernel<")[1].split(">")[0]
        agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(key, r["Counter_Name"])] += 1
    for key, d in agg.items():
        print(tag, key, {c: round(v / max(n[(key, c)], 1)) for c, v in d.items()})
PY
exit $rc
