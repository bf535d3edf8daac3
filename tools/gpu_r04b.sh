#!/usr/bin/env bash
# GPU (round 4, call B): per-phase stamps of the deep-level register-streamed
# convs, SQ counters of the same, then C4 (profile + per-op PMC + per-shard
# batches) and C5 (whole vs chunked pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r04b}
OUHIP_LIB=$PWD/open_universe_amd/variants/libouhip_stamps.so timeout -k 10 300 python3 tools/conv_bench.py \
    --layer L4k3 --tile 16384 --stamps --reps 20 > $O/stamps_$TAG.txt 2>&1 &&
OUHIP_LIB=$PWD/open_universe_amd/variants/libouhip_stamps.so timeout -k 10 300 python3 tools/conv_bench.py \
    --layer L4k5,GI,U3,L3k3 --stamps --reps 20 >> $O/stamps_$TAG.txt 2>&1 || { tail -20 $O/stamps_$TAG.txt; exit 1; }
cat $O/stamps_$TAG.txt
cd /tmp
P="timeout -s KILL 90 rocprofv3 --output-format csv"
$P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
    -d $GRAFT_REPO_ROOT/$O/cpmc1_$TAG -o pmc -- python3 $GRAFT_REPO_ROOT/tools/conv_bench.py --layer L4k3 --tile 16384 --reps 20 \
    > $GRAFT_REPO_ROOT/$O/cpmc1_$TAG.log 2>&1 || echo "pmc pass 1 failed"
$P --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU \
    -d $GRAFT_REPO_ROOT/$O/cpmc2_$TAG -o pmc -- python3 $GRAFT_REPO_ROOT/tools/conv_bench.py --layer L4k3 --tile 16384 --reps 20 \
    > $GRAFT_REPO_ROOT/$O/cpmc2_$TAG.log 2>&1 || echo "pmc pass 2 failed"
cd $GRAFT_REPO_ROOT
python3 tools/pmc_avg.py "$(find $O/cpmc1_$TAG -name '*counter_collection.csv' | head -n1)" conv_rkernel > $O/cpmc_$TAG.txt 2>&1
python3 tools/pmc_avg.py "$(find $O/cpmc2_$TAG -name '*counter_collection.csv' | head -n1)" conv_rkernel >> $O/cpmc_$TAG.txt 2>&1
cat $O/cpmc_$TAG.txt
# first-step schedule: mel on its own lane + reassociated st sum (default) vs mel on the st lane
for v in base:OUHIP_MEL_LANE=2 st:OUHIP_MEL_LANE=1 base2:OUHIP_MEL_LANE=2; do
  n=${v%%:*}; e=${v#*:}
  env $e OUHIP_TUNE_CACHE=$O/tune_${TAG}_c2.json timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline \
      --no-f32-pass --no-queued --traffic-json "" > $O/ab_${TAG}_$n.json 2> $O/ab_${TAG}_$n.err || { tail -5 $O/ab_${TAG}_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/ab_${TAG}_$n.json')); print('$n', d['value'], d['ms_per_step'], d['profile'])"
done
OUHIP_TUNE_CACHE=$O/tune_${TAG}_c2.json timeout -k 10 300 python3 tools/critical_path.py --config c2 --reps 3 --ops \
    --out $O/cp_$TAG.json > $O/cp_$TAG.txt 2>&1 || { tail -20 $O/cp_$TAG.txt; exit 1; }
head -45 $O/cp_$TAG.txt
# C4 profile (kernel trace + PMC of this library) and per-op table
bash tools/gpu_profile.sh ${TAG}_c4 c4 --steps 4 --warmup 1 --no-f32-pass --no-queued || exit 1
bash tools/gpu_level_pmc.sh ${TAG}_c4lv c4 || exit 1
for b in 16 8 4; do
  timeout -k 10 300 python3 bench.py --config c4 --batch $b --steps 4 --warmup 1 --no-f32-pass --no-cpu-baseline \
      --traffic-json "" > $O/bench_${TAG}_c4_b$b.json 2> $O/bench_${TAG}_c4_b$b.err || { tail -5 $O/bench_${TAG}_c4_b$b.err; exit 1; }
done
for c in 0 1; do
  OUHIP_CHUNK=$c timeout -k 10 300 python3 bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline \
      > $O/bench_${TAG}_c5_chunk$c.json 2> $O/bench_${TAG}_c5_chunk$c.err || { tail -5 $O/bench_${TAG}_c5_chunk$c.err; exit 1; }
done
for f in $O/bench_${TAG}_c4_b*.json $O/bench_${TAG}_c5_chunk*.json; do echo "$f"; python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d.get('profile'))"; done
