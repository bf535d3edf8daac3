#!/usr/bin/env bash
# GPU (round 4, call D): kernel-argument prefetch in the conv / block kernels.
# Tests (conv tiles, fused blocks, chunked pass, layer parity, C3 real shape,
# PP24 range fallback), conv A/B and C2 bench A/B against the r04c library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r04d}
V=$PWD/open_universe_amd/variants
NEW=$PWD/open_universe_amd/libouhip.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_conv_tiles.py tests/test_gpu_block.py tests/test_gpu_chunked.py tests/test_gpu_parity.py \
    "tests/test_gpu_parity_sizes.py::test_c3_real_shape_item0_vs_oracle" \
    "tests/test_gpu_parity_sizes.py::test_full_width_pp24_enhance" \
    "tests/test_gpu_parity_sizes.py::test_c2_size_enhance_vs_oracle" \
    > $O/tests_$TAG.log 2>&1 || { tail -30 $O/tests_$TAG.log; exit 1; }
tail -3 $O/tests_$TAG.log
for lib in new r04c; do
  L=$NEW; [ $lib = r04c ] && L=$V/libouhip_r04c.so
  OUHIP_LIB=$L timeout -k 10 200 python3 tools/conv_bench.py --layer L4k3,L4k5,GI,U3,L3k3,L3k5,D2,U2,L2k3,L1k3 --reps 20 \
      > $O/cb_${TAG}_$lib.txt 2>&1 || { tail -5 $O/cb_${TAG}_$lib.txt; exit 1; }
done
for f in new r04c; do echo "== $f"; grep -v amdgpu $O/cb_${TAG}_$f.txt | awk '{print $1, $5, $6, $7}'; done
ab() {   # ab NAME LIB [ENV...]
  local name=$1 lib=$2; shift 2
  env "$@" OUHIP_LIB=$lib OUHIP_TUNE_CACHE=$O/tune_${TAG}_$(basename $lib .so).json timeout -k 10 200 \
      python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32-pass --no-queued \
      --traffic-json "" > $O/ab_${TAG}_$name.json 2> $O/ab_${TAG}_$name.err || { tail -5 $O/ab_${TAG}_$name.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/ab_${TAG}_$name.json')); print('$name', d['value'], d['ms_per_step'], d['profile'])"
}
ab new $NEW && ab r04c $V/libouhip_r04c.so && ab new2 $NEW && ab r04c2 $V/libouhip_r04c.so || exit 1
