#!/usr/bin/env bash
# GPU (round 4, call C): conv_rkernel staging (buffer loads, incremental
# items) + epilogue loads ahead of the K-split reduction.  Tile tests, stamps
# of the new kernel, conv A/B and C2 bench A/B against the r04a library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r04c}
V=$PWD/open_universe_amd/variants
NEW=$PWD/open_universe_amd/libouhip.so
timeout -k 10 420 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_conv_tiles.py tests/test_gpu_chunked.py \
    "tests/test_gpu_parity.py::test_same_conv_layer" "tests/test_gpu_parity.py::test_down_conv_layer" \
    "tests/test_gpu_parity.py::test_up_conv_layer" \
    "tests/test_gpu_parity_sizes.py::test_c2_size_enhance_vs_oracle" \
    > $O/tests_$TAG.log 2>&1 || { tail -30 $O/tests_$TAG.log; exit 1; }
tail -3 $O/tests_$TAG.log
OUHIP_LIB=$V/libouhip_stamps.so timeout -k 10 300 python3 tools/conv_bench.py \
    --layer L4k3 --tile 16384 --stamps --reps 20 > $O/stamps_$TAG.txt 2>&1 &&
for L in L4k5:16384 GI:16386 U3:16386 L3k3:16386 D2:16386 ST0:16384; do
  OUHIP_LIB=$V/libouhip_stamps.so timeout -k 10 300 python3 tools/conv_bench.py \
      --layer ${L%%:*} --tile ${L##*:} --stamps --reps 20 >> $O/stamps_$TAG.txt 2>&1 || exit 1
done
grep -v amdgpu $O/stamps_$TAG.txt
for lib in new r04a; do
  L=$NEW; [ $lib = r04a ] && L=$V/libouhip_r04a.so
  OUHIP_LIB=$L timeout -k 10 200 python3 tools/conv_bench.py --layer L4k3,L4k5,GI,U3,L3k3,L3k5,D3,D2,U2,ST0,ST1 --reps 20 \
      > $O/cb_${TAG}_$lib.txt 2>&1 || { tail -5 $O/cb_${TAG}_$lib.txt; exit 1; }
done
grep -v amdgpu $O/cb_${TAG}_new.txt $O/cb_${TAG}_r04a.txt | cut -c1-200
ab() {   # ab NAME LIB [ENV...]
  local name=$1 lib=$2; shift 2
  env "$@" OUHIP_LIB=$lib OUHIP_TUNE_CACHE=$O/tune_${TAG}_$(basename $lib .so).json timeout -k 10 200 \
      python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32-pass --no-queued \
      --traffic-json "" > $O/ab_${TAG}_$name.json 2> $O/ab_${TAG}_$name.err || { tail -5 $O/ab_${TAG}_$name.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/ab_${TAG}_$name.json')); print('$name', d['value'], d['ms_per_step'], d['profile'])"
}
ab new $NEW && ab r04a $V/libouhip_r04a.so && ab new2 $NEW && ab r04a2 $V/libouhip_r04a.so || exit 1
