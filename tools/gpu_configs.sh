#!/usr/bin/env bash
# Measure the non-headline BASELINE configs (c3, c4, c5) with bench.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${1:-cfg}
for c in ${CONFIGS:-c5 c3 c4}; do
  timeout -k 10 400 python bench.py --config $c --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline \
      > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err || { echo "config $c failed"; tail -5 gpurun_out/bench_${TAG}_$c.err; exit 1; }
  cat gpurun_out/bench_${TAG}_$c.json
done
