#!/usr/bin/env bash
# GPU (round 4, call E): m-major workgroup order for large batched inputs (C4),
# A/B at C4 with the per-op table; C2 unchanged check.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r04e}
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_conv_tiles.py "tests/test_gpu_parity_sizes.py::test_c4_real_shape_damped_split_f16_item0_vs_oracle" \
    > $O/tests_$TAG.log 2>&1 || { tail -30 $O/tests_$TAG.log; exit 1; }
tail -2 $O/tests_$TAG.log
for v in maj1:1 maj0:0; do
  n=${v%%:*}; e=${v#*:}
  OUHIP_MMAJOR=$e OUHIP_TUNE_CACHE=$O/tune_${TAG}_c4.json timeout -k 10 400 python3 bench.py --config c4 --steps 3 --warmup 1 \
      --no-cpu-baseline --no-f32-pass --dump-ops $O/ops_${TAG}_$n.json --traffic-json "" > $O/bench_${TAG}_$n.json 2> $O/bench_${TAG}_$n.err \
      || { tail -5 $O/bench_${TAG}_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_${TAG}_$n.json')); print('$n', d['value'], d['ms_per_step'], d['profile'])"
done
OUHIP_MMAJOR=1 OUHIP_TUNE_CACHE=$O/tune_${TAG}_c4.json bash tools/gpu_level_pmc.sh ${TAG}_lv c4 || exit 1
