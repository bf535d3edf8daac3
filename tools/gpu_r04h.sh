#!/usr/bin/env bash
# GPU (round 4, call H): register-streamed weight-ring depth A/B (8 / 12 / 16
# steps) on the deep-level convs and the C2 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r04h}
V=$PWD/open_universe_amd/variants
NEW=$PWD/open_universe_amd/libouhip.so
for v in r12:$NEW r16:$V/libouhip_ring16.so r8:$V/libouhip_ring8.so; do
  n=${v%%:*}; L=${v#*:}
  OUHIP_LIB=$L timeout -k 10 200 python3 tools/conv_bench.py --layer L4k3,L4k5,GI,U3,L3k3,L3k5,D2 --reps 20 \
      > $O/cb_${TAG}_$n.txt 2>&1 || { tail -5 $O/cb_${TAG}_$n.txt; exit 1; }
  echo "== $n"; grep -v amdgpu $O/cb_${TAG}_$n.txt | awk '{print $1, $5, $6, $7}'
done
for v in r12:$NEW r16:$V/libouhip_ring16.so r12b:$NEW r16b:$V/libouhip_ring16.so; do
  n=${v%%:*}; L=${v#*:}
  OUHIP_LIB=$L OUHIP_TUNE_CACHE=$O/tune_${TAG}_$(basename $L .so).json timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 \
      --no-cpu-baseline --no-f32-pass --no-queued --traffic-json "" > $O/ab_${TAG}_$n.json 2> $O/ab_${TAG}_$n.err \
      || { tail -5 $O/ab_${TAG}_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/ab_${TAG}_$n.json')); print('c2 $n', d['value'], d['ms_per_step'], d['profile'])"
done
