#!/usr/bin/env bash
# GPU A/B of two libouhip builds: conv_bench on the deep-level layers and
# the C2 bench line with each.  Usage: tools/gpu_ab.sh TAG LIB_B [LAYERS]
#   (A = the in-tree libouhip.so; LIB_B e.g. open_universe_amd/variants/libouhip_noxcd.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out
mkdir -p $O
export PYTHONUNBUFFERED=1
TAG=$1; LB=$2; LAYERS=${3:-L4k3,L4k5,L3k3,L3k5,GI,U3,U2,D2,D3}
BENCH="python -u bench.py --no-cpu-baseline --no-queued --no-f32-pass --steps 10 --warmup 2"
timeout -k 10 300 python -u tools/conv_bench.py --layer $LAYERS > $O/ab_conv_A_$TAG.txt 2>&1 || exit $?
OUHIP_LIB=$PWD/$LB timeout -k 10 300 python -u tools/conv_bench.py --layer $LAYERS > $O/ab_conv_B_$TAG.txt 2>&1 || exit $?
timeout -k 10 300 $BENCH > $O/ab_bench_A_$TAG.json 2> $O/ab_bench_A_$TAG.err || exit $?
OUHIP_LIB=$PWD/$LB timeout -k 10 300 $BENCH > $O/ab_bench_B_$TAG.json 2> $O/ab_bench_B_$TAG.err || exit $?
timeout -k 10 300 $BENCH > $O/ab_bench_A2_$TAG.json 2> $O/ab_bench_A2_$TAG.err || exit $?
OUHIP_GRU_FLAGS=${AB_GRU_FLAGS:-257} timeout -k 10 300 $BENCH > $O/ab_bench_Ag_$TAG.json 2> $O/ab_bench_Ag_$TAG.err || exit $?
GRU_FLAGS=1,257,513 timeout -k 10 200 python -u tools/gru_bench.py > $O/ab_grub_$TAG.log 2>&1 || exit $?
