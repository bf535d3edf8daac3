#!/usr/bin/env bash
# GPU (round 4, call I): conditions signalled right after conv1, score decoder
# waits after its up conv.  Parity tests, lane timeline, C2 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r04i}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    tests/test_gpu_chunked.py "tests/test_gpu_parity_sizes.py::test_c2_size_enhance_vs_oracle" \
    "tests/test_gpu_parity_sizes.py::test_full_width_orig16_enhance_8_and_60_steps" \
    "tests/test_gpu_parity_sizes.py::test_enhance_many_equals_sequential_enhance" \
    > $O/tests_$TAG.log 2>&1 || { tail -30 $O/tests_$TAG.log; exit 1; }
tail -2 $O/tests_$TAG.log
export OUHIP_TUNE_CACHE=$O/tune_${TAG}.json
timeout -k 10 300 python3 tools/critical_path.py --config c2 --reps 3 --ops --out $O/cp_$TAG.json > $O/cp_$TAG.txt 2>&1 || { tail -20 $O/cp_$TAG.txt; exit 1; }
grep -v amdgpu $O/cp_$TAG.txt | head -48
for n in a b c; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32-pass --no-queued --traffic-json "" \
      > $O/ab_${TAG}_$n.json 2> $O/ab_${TAG}_$n.err || { tail -5 $O/ab_${TAG}_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/ab_${TAG}_$n.json')); print('c2 $n', d['value'], d['ms_per_step'], d['profile'])"
done
