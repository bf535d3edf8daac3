#!/usr/bin/env bash
# GPU: C2 bench under lane / replay variants (st_convs lane, eager replay),
# then the fused-block decomposition.  Usage: tools/gpu_lanes_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
export PYTHONUNBUFFERED=1
TAG=${1:-lanes}
B="python -u bench.py --no-cpu-baseline --no-queued --no-f32-pass --steps 10 --warmup 2"
timeout -k 10 300 $B > $O/la_base_$TAG.json 2> $O/la_base_$TAG.err || exit $?
OUHIP_ST_LANE=0 timeout -k 10 300 $B > $O/la_st0_$TAG.json 2> $O/la_st0_$TAG.err || exit $?
OUHIP_GRAPH=0 timeout -k 10 300 $B > $O/la_eager_$TAG.json 2> $O/la_eager_$TAG.err || exit $?
timeout -k 10 300 $B > $O/la_base2_$TAG.json 2> $O/la_base2_$TAG.err || exit $?
bash tools/gpu_block_dbg.sh $TAG > /dev/null
