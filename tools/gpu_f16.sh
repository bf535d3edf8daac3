#!/usr/bin/env bash
# GPU tests, then the c2 bench (split-f16 default) and the c5 bench (fp16 conv operands).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/f16_pytest.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err &&
timeout -k 10 600 python bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err
rc=$?
tail -15 gpurun_out/f16_pytest.log; cat gpurun_out/bench_c2.json gpurun_out/bench_c5.json; tail -3 gpurun_out/bench_c5.err
exit $rc
