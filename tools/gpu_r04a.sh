#!/usr/bin/env bash
# GPU (round 4, call A): targeted GPU tests (incl. every conv tile), the
# register-streamed conv A/B (new scalar-indexed K loop vs the previous one),
# C2 bench A/B, then the C2 profile (kernel trace + PMC of this library), the
# per-op PMC table and the lane timeline of C2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r04a}
V=$PWD/open_universe_amd/variants
timeout -k 10 420 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_conv_tiles.py \
    "tests/test_gpu_parity.py::test_gru_ws_zeroed_short_launches_back_to_back" \
    "tests/test_gpu_parity.py::test_same_conv_layer" "tests/test_gpu_parity.py::test_down_conv_layer" \
    "tests/test_gpu_parity.py::test_up_conv_layer" \
    "tests/test_gpu_parity_sizes.py::test_c2_size_enhance_vs_oracle" \
    > $O/tests_$TAG.log 2>&1 || { tail -30 $O/tests_$TAG.log; exit 1; }
tail -3 $O/tests_$TAG.log
for lib in new old; do
  L=$PWD/open_universe_amd/libouhip.so; [ $lib = old ] && L=$V/libouhip_oldrk.so
  OUHIP_LIB=$L timeout -k 10 200 python3 tools/conv_bench.py --layer L4k3,L4k5,GI,U3,L3k3,D3,D2,ST0 --reps 20 \
      > $O/cb_${TAG}_$lib.txt 2>&1 || { tail -5 $O/cb_${TAG}_$lib.txt; exit 1; }
done
head -20 $O/cb_${TAG}_new.txt $O/cb_${TAG}_old.txt
ab() {   # ab NAME LIB [ENV...]
  local name=$1 lib=$2; shift 2
  env "$@" OUHIP_LIB=$lib OUHIP_TUNE_CACHE=$O/tune_${TAG}_$(basename $lib .so).json timeout -k 10 200 \
      python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32-pass --no-queued \
      --traffic-json "" > $O/ab_${TAG}_$name.json 2> $O/ab_${TAG}_$name.err || { tail -5 $O/ab_${TAG}_$name.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/ab_${TAG}_$name.json')); print('$name', d['value'], d['ms_per_step'], d['profile'])"
}
NEW=$PWD/open_universe_amd/libouhip.so
ab new $NEW && ab old $V/libouhip_oldrk.so && ab new2 $NEW && ab mel2 $NEW OUHIP_MEL_LANE=2 &&
ab after $NEW OUHIP_SCORE_AFTER_CENC=1 && ab both $NEW OUHIP_MEL_LANE=2 OUHIP_SCORE_AFTER_CENC=1 && ab new3 $NEW || exit 1
export OUHIP_TUNE_CACHE=$O/tune_${TAG}_libouhip.json
timeout -k 10 300 python3 tools/critical_path.py --config c2 --reps 3 --ops --out $O/cp_$TAG.json > $O/cp_$TAG.txt 2>&1 || { tail -20 $O/cp_$TAG.txt; exit 1; }
head -70 $O/cp_$TAG.txt
OUHIP_MEL_LANE=2 OUHIP_SCORE_AFTER_CENC=1 timeout -k 10 300 python3 tools/critical_path.py --config c2 --reps 3 --ops \
    --out $O/cp_${TAG}_both.json > $O/cp_${TAG}_both.txt 2>&1 || { tail -20 $O/cp_${TAG}_both.txt; exit 1; }
head -50 $O/cp_${TAG}_both.txt
unset OUHIP_TUNE_CACHE
bash tools/gpu_profile.sh $TAG c2 || exit 1
