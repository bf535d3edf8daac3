#!/usr/bin/env bash
# split-f16 bring-up: conv tile tests (both precisions), parity, bench both ways.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_conv_tiles.py > gpurun_out/split_tiles.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/split_pytest.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --dump-ops gpurun_out/ops_split.json > gpurun_out/bench_split.json 2> gpurun_out/bench_split.err &&
OUHIP_CONV_PREC=f32 timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_f32.json 2> gpurun_out/bench_f32.err
rc=$?
tail -5 gpurun_out/split_tiles.log; tail -15 gpurun_out/split_pytest.log; cat gpurun_out/bench_split.json gpurun_out/bench_f32.json; tail -3 gpurun_out/bench_split.err
exit $rc
