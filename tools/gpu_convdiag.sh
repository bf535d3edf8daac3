#!/usr/bin/env bash
# GPU: per-layer ou_conv tile sweep of the deep PP16 layers with the
# register-streamed diagnostics (no input loads / no K loop), and the fused
# block microbenchmark.  Outputs under gpurun_out/convdiag_TAG.txt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-run}
export PYTHONUNBUFFERED=1
timeout -k 10 500 python tools/conv_bench.py --layer ${LAYERS:-L4k3,L4k5,L3k3,L3k5,U3,GI,U2,U1,D2,D3} --rdiag --reps 30 \
    > gpurun_out/convdiag_$TAG.txt 2>&1 &&
timeout -k 10 300 python tools/block_bench.py --reps 30 --dbg 1,2,4,3 >> gpurun_out/convdiag_$TAG.txt 2>&1
rc=$?
cat gpurun_out/convdiag_$TAG.txt
exit $rc
