#!/usr/bin/env bash
# GPU (round 4, call A): the new GPU tests, then the C2 profile (kernel trace +
# PMC of this library) and the per-op PMC table of C2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r04a}
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
    "tests/test_gpu_parity.py::test_gru_ws_zeroed_short_launches_back_to_back" \
    "tests/test_gpu_parity.py::test_gru_layer" \
    "tests/test_gpu_parity_sizes.py::test_c3_real_shape_item0_vs_oracle" \
    "tests/test_gpu_parity_sizes.py::test_full_width_pp24_enhance" \
    "tests/test_gpu_audio.py::test_enhance_cli_outputs_independent_of_world_size" \
    > $O/tests_$TAG.log 2>&1 || { tail -30 $O/tests_$TAG.log; exit 1; }
tail -3 $O/tests_$TAG.log
bash tools/gpu_profile.sh $TAG c2 || exit 1
bash tools/gpu_level_pmc.sh ${TAG}_lv c2 || exit 1
timeout -k 10 300 python3 tools/critical_path.py --config c2 --reps 3 --ops --out $O/cp_$TAG.json > $O/cp_$TAG.txt 2>&1 || { tail -20 $O/cp_$TAG.txt; exit 1; }
head -60 $O/cp_$TAG.txt
