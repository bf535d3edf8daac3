#!/usr/bin/env bash
# PMC passes over single conv configurations (tools/conv_bench.py).
# Usage: tools/gpu_convpmc.sh TAG "LAYER:TILE LAYER:TILE ..."
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=$1
O="$ROOT/gpurun_out/convpmc_$TAG"
mkdir -p "$O"
export TMPDIR=/tmp
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
B="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
rc=0
for lt in $2; do
  l=${lt%%:*}; t=${lt##*:}
  for p in A B; do
    cd /tmp
    timeout -k 10 300 rocprofv3 --pmc ${!p} --output-format csv -d "$O/${l}_t${t}_$p" -o pmc -- \
      python3 "$ROOT/tools/conv_bench.py" --layer "$l" --tile "$t" --reps 30 > "$O/${l}_t${t}_$p.log" 2>&1 || { rc=$?; break 2; }
    python3 "$ROOT/tools/pmc_avg.py" "$(find "$O/${l}_t${t}_$p" -name '*counter_collection.csv' | head -n1)" >> "$O/summary.txt"
  done
  cat "$O/${l}_t${t}_A.log" | tail -1 >> "$O/summary.txt"
done
cat "$O/summary.txt"
exit $rc
