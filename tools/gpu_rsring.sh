#!/usr/bin/env bash
# GPU: register-streamed conv ring depth (OU_RS_RING variants): conv_bench on
# the deep layers and the C2 bench with each library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
export PYTHONUNBUFFERED=1
TAG=${1:-rs}; shift
L=L4k3,L4k5,GI,U3,D3,L3k3,ST0,ST1
B="python -u bench.py --no-cpu-baseline --no-queued --no-f32-pass --steps 10 --warmup 2"
timeout -k 10 300 python -u tools/conv_bench.py --layer $L 2>/dev/null | grep -v amdgpu > $O/rs_conv_base_$TAG.txt || exit $?
timeout -k 10 300 $B > $O/rs_bench_base_$TAG.json 2> $O/rs_bench_base_$TAG.err || exit $?
for v in "$@"; do
  OUHIP_LIB=$PWD/open_universe_amd/variants/libouhip_$v.so timeout -k 10 300 python -u tools/conv_bench.py --layer $L 2>/dev/null | grep -v amdgpu > $O/rs_conv_${v}_$TAG.txt || exit $?
  OUHIP_LIB=$PWD/open_universe_amd/variants/libouhip_$v.so timeout -k 10 300 $B > $O/rs_bench_${v}_$TAG.json 2> $O/rs_bench_${v}_$TAG.err || exit $?
done
