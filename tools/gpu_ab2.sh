#!/usr/bin/env bash
# GPU: correctness subset, then A/B of the pipelined GRU poll (flags bit10)
# and the channel-major up-conv rows (OUHIP_UP_CM) on the C2 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
export PYTHONUNBUFFERED=1
TAG=${1:-ab2}
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_conv_tiles.py tests/test_gpu_parity.py tests/test_gpu_chunked.py > $O/ab2_tests_$TAG.log 2>&1 || { tail -30 $O/ab2_tests_$TAG.log; exit 1; }
tail -2 $O/ab2_tests_$TAG.log
GRU_FLAGS=1,1025,1,1025 timeout -k 10 200 python -u tools/gru_bench.py > $O/ab2_grub_$TAG.log 2>&1 || exit $?
B="python -u bench.py --no-cpu-baseline --no-queued --no-f32-pass --steps 10 --warmup 2"
timeout -k 10 300 $B > $O/ab2_base_$TAG.json 2> $O/ab2_base_$TAG.err || exit $?
OUHIP_GRU_FLAGS=1025 timeout -k 10 300 $B > $O/ab2_pipe_$TAG.json 2> $O/ab2_pipe_$TAG.err || exit $?
OUHIP_UP_CM=0 timeout -k 10 300 $B > $O/ab2_pm_$TAG.json 2> $O/ab2_pm_$TAG.err || exit $?
timeout -k 10 300 $B > $O/ab2_base2_$TAG.json 2> $O/ab2_base2_$TAG.err || exit $?
