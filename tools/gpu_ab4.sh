#!/usr/bin/env bash
# GPU: C2 bench, up convs channel-major from rate 3 (default) vs from rate 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
export PYTHONUNBUFFERED=1
TAG=${1:-ab4}
B="python -u bench.py --no-cpu-baseline --no-queued --no-f32-pass --steps 10 --warmup 2"
timeout -k 10 300 $B > $O/ab4_r3_$TAG.json 2> $O/ab4_r3_$TAG.err || exit $?
OUHIP_UP_CM_MIN_RATE=2 timeout -k 10 300 $B > $O/ab4_r2_$TAG.json 2> $O/ab4_r2_$TAG.err || exit $?
timeout -k 10 300 $B > $O/ab4_r3b_$TAG.json 2> $O/ab4_r3b_$TAG.err || exit $?
OUHIP_UP_CM_MIN_RATE=2 timeout -k 10 300 $B > $O/ab4_r2b_$TAG.json 2> $O/ab4_r2b_$TAG.err || exit $?
