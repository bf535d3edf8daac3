#!/usr/bin/env bash
# GPU (round 4, call G): fused-block staging through a buffer resource.  The
# whole GPU suite, then C2 / C4 A/B against the r04f library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r04g}
V=$PWD/open_universe_amd/variants
NEW=$PWD/open_universe_amd/libouhip.so
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
    > $O/tests_$TAG.log 2>&1 || { tail -30 $O/tests_$TAG.log; exit 1; }
tail -2 $O/tests_$TAG.log
for v in new:$NEW r04f:$V/libouhip_r04f.so new2:$NEW r04f2:$V/libouhip_r04f.so; do
  n=${v%%:*}; L=${v#*:}
  OUHIP_LIB=$L OUHIP_TUNE_CACHE=$O/tune_${TAG}_c2_$(basename $L .so).json timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 \
      --no-cpu-baseline --no-f32-pass --no-queued --traffic-json "" > $O/ab_${TAG}_$n.json 2> $O/ab_${TAG}_$n.err \
      || { tail -5 $O/ab_${TAG}_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/ab_${TAG}_$n.json')); print('c2 $n', d['value'], d['ms_per_step'], d['profile'])"
done
for v in new:$NEW r04f:$V/libouhip_r04f.so; do
  n=${v%%:*}; L=${v#*:}
  OUHIP_LIB=$L OUHIP_TUNE_CACHE=$O/tune_${TAG}_c4_$n.json timeout -k 10 400 python3 bench.py --config c4 --steps 3 --warmup 1 \
      --no-cpu-baseline --no-f32-pass --traffic-json "" > $O/bench_${TAG}_c4_$n.json 2> $O/bench_${TAG}_c4_$n.err \
      || { tail -5 $O/bench_${TAG}_c4_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_${TAG}_c4_$n.json')); print('c4 $n', d['value'], d['ms_per_step'], d['profile'])"
done
