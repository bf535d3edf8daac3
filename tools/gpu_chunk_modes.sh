#!/usr/bin/env bash
# GPU: the C2 bench unchunked / chunked under whole-graph, segmented-graph
# and eager replay and hardware-queue counts (experiments for the chunked
# score pass).  Outputs gpurun_out/cm_*.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out
mkdir -p $O
export PYTHONUNBUFFERED=1
B="python -u bench.py --no-cpu-baseline --no-queued --no-f32-pass --no-profile --steps 10 --warmup 2"
run() { local tag=$1; shift; env "$@" timeout -k 10 240 $B > $O/cm_$tag.json 2> $O/cm_$tag.err; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chunked.py tests/test_gpu_block.py > $O/cm_tests.log 2>&1 || exit $?
run plain OUHIP_CHUNK=0 || exit $?
run chunk OUHIP_CHUNK=1 || exit $?
run plain_seg OUHIP_CHUNK=0 OUHIP_GRAPH_MODE=seg || exit $?
run chunk_seg OUHIP_CHUNK=1 OUHIP_GRAPH_MODE=seg || exit $?
run chunk_q8 OUHIP_CHUNK=1 GPU_MAX_HW_QUEUES=8 || exit $?
run chunk_seg_q8 OUHIP_CHUNK=1 OUHIP_GRAPH_MODE=seg GPU_MAX_HW_QUEUES=8 || exit $?
