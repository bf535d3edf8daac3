#!/usr/bin/env bash
# GPU: fused-block time decomposition (tools/block_bench.py diagnostic masks:
# 1 no input loads, 2 no MFMA stages, 4 no output pass, combinations).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/block_bench.py --levels ${LEVELS:-0,1,2} --dbg ${DBG:-1,2,4,3,6,7} > gpurun_out/block_dbg_${1:-run}.txt 2>&1
rc=$?; cat gpurun_out/block_dbg_${1:-run}.txt; exit $rc
