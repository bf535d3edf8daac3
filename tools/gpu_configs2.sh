#!/usr/bin/env bash
# GPU: the other BASELINE configs with the warm-up / step counts of the
# committed profiles (C1 20/3, C5 5/3, C3 and C4 3/1 without the f32 leg).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
export PYTHONUNBUFFERED=1
TAG=${1:-cfg}
run() { local c=$1; shift; timeout -k 10 500 python -u bench.py --config $c --no-cpu-baseline "$@" > $O/bench_${TAG}_$c.json 2> $O/bench_${TAG}_$c.err || { echo "config $c failed"; tail -3 $O/bench_${TAG}_$c.err; return 1; }; }
run c1 --steps 20 --warmup 3 || exit 1
run c5 --steps 5 --warmup 3 || exit 1
run c4 --steps 3 --warmup 1 --no-f32-pass --no-queued || exit 1
run c3 --steps 3 --warmup 1 --no-f32-pass --no-queued || exit 1
