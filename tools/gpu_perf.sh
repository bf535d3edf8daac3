#!/usr/bin/env bash
# GPU tests + bench with per-op dump.  Usage: tools/gpu_perf.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-run}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_$TAG.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 10 --warmup 2 ${BENCH_ARGS:-} --dump-ops gpurun_out/ops_$TAG.json > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?
tail -3 gpurun_out/pytest_gpu_$TAG.log; tail -2 gpurun_out/bench_$TAG.err; cat gpurun_out/bench_$TAG.json
exit $rc
