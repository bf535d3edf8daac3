#!/usr/bin/env bash
# GPU: fused-block early weight ring A/B (variant early0), block tests, and the
# C2 bench with / without the mel branch on the st_conv lane (OUHIP_MEL_LANE).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
export PYTHONUNBUFFERED=1
TAG=${1:-ab3}
bash tools/gpu_block_variants.sh $TAG early0 > /dev/null || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_block.py tests/test_gpu_parity.py > $O/ab3_tests_$TAG.log 2>&1 || { tail -20 $O/ab3_tests_$TAG.log; exit 1; }
B="python -u bench.py --no-cpu-baseline --no-queued --no-f32-pass --steps 10 --warmup 2"
timeout -k 10 300 $B > $O/ab3_base_$TAG.json 2> $O/ab3_base_$TAG.err || exit $?
OUHIP_LIB=$PWD/open_universe_amd/variants/libouhip_early0.so timeout -k 10 300 $B > $O/ab3_e0_$TAG.json 2> $O/ab3_e0_$TAG.err || exit $?
OUHIP_MEL_LANE=0 timeout -k 10 300 $B > $O/ab3_mel0_$TAG.json 2> $O/ab3_mel0_$TAG.err || exit $?
timeout -k 10 300 $B > $O/ab3_base2_$TAG.json 2> $O/ab3_base2_$TAG.err || exit $?
