#!/usr/bin/env bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_tiles.py > gpurun_out/convtiles_tiles.log 2>&1 &&
timeout -k 10 500 python tools/conv_bench.py > gpurun_out/convtiles_cb.log 2>&1
rc=$?
tail -3 gpurun_out/convtiles_tiles.log; cat gpurun_out/convtiles_cb.log
exit $rc
