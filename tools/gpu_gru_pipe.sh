#!/usr/bin/env bash
# GPU: GRU poll variants on a variant library (OUHIP_LIB), then the C2 bench
# with the variant flags.  Usage: tools/gpu_gru_pipe.sh LIB FLAGS_LIST BENCH_FLAGS
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
export PYTHONUNBUFFERED=1 OUHIP_LIB=$PWD/$1
GRU_FLAGS=$2 timeout -k 10 200 python -u tools/gru_bench.py > $O/grub_pipe.log 2>&1 || exit $?
OUHIP_GRU_FLAGS=$3 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-queued --no-f32-pass --steps 10 --warmup 2 > $O/bench_pipe.json 2> $O/bench_pipe.err || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-queued --no-f32-pass --steps 10 --warmup 2 > $O/bench_pipe_base.json 2> $O/bench_pipe_base.err || exit $?
