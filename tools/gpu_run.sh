#!/usr/bin/env bash
# The one runner for GPU-box work (gpurun -- 'bash tools/gpu_run.sh TAG STEP...').
# Every step runs under its own time limit; the first failing step ends the
# call (no retries).  Outputs go to gpurun_out/*_TAG*.
#
#   tests            the whole `pytest -m gpu` suite
#   tests:FILE[::T]  one test file / test
#   profile:CFG      tools/gpu_profile.sh (bench line, kernel trace, FETCH/WRITE PMC passes)
#   levels:CFG       tools/gpu_level_pmc.sh (per-op conv-stack table)
#   bench:CFG        bench.py --config CFG, default arguments (the driver's line)
#   benchpmc:CFG     profile:CFG, then bench:CFG quoting `traffic` from that PMC summary
#   shards           C4 at the per-rank batches of 2/4/8 GPUs (B = 16, 8, 4)
#   c4u              C4 on the undamped synthetic weights (exponents widen in the warm-up)
#   critical         tools/critical_path.py --config c2 (lane timeline, first step)
#   ab:VAR=[A,]B     C2 bench with VAR=A / B / A / B (A defaults to 0; same box, alternating)
#   ablib:NAME       C2 bench, in-tree libouhip.so vs variants/libouhip_NAME.so (3 pairs)
#   convlib:NAME     tools/conv_bench.py deep-level layers, in-tree library vs the variant
#   convsplit[:L,..] tools/conv_bench.py --split: the split-image kernel on the deep-level layers
#   convsplitlib:A,B the same on the k3 layers, in-tree library then variants A, B (stamps: --sstamps)
#   fir:CFG          tools/fir_bench.py: folded vs FIR-applied rate-change convs at CFG
#   sqfir:CFG/L/T    SQ counters (two rocprofv3 --pmc passes) of FIR layer L on tile T
#   sqconv:L/T       the same for tools/conv_bench.py layer L on conv_kernel tile T
#   sqblock:LEVEL    the same for a PP24 fused block at C4's batch (tools/block_bench.py)
#   firtile:CFG/L/T1,T2  FIR layer L timed on each listed tile
#
#   e.g. tools/gpu_run.sh r04k profile:c2 critical bench:c1 bench:c3 bench:c5
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=$1; shift
O="$ROOT/gpurun_out"; mkdir -p "$O"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
line() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['unit'], d['ms_per_step'], d.get('profile'), d.get('fallbacks'))" "$1"; }
bench() {   # bench OUT LIMIT ARGS...
    local out=$1 lim=$2; shift 2
    timeout -k 10 "$lim" python3 bench.py "$@" > "$out.json" 2> "$out.err" || { tail -20 "$out.err"; return 1; }
    line "$out.json"
}
for step in "$@"; do
    name=${step%%:*}; arg=${step#*:}; [ "$arg" = "$step" ] && arg=""
    echo "== $step"
    case $name in
    tests)
        timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${arg:-tests} \
            > "$O/tests_$TAG.log" 2>&1 || { tail -40 "$O/tests_$TAG.log"; exit 1; }
        tail -3 "$O/tests_$TAG.log" ;;
    profile)
        if [ "$arg" = c2 ]; then bash tools/gpu_profile.sh "$TAG" c2 || exit 1
        else bash tools/gpu_profile.sh "${TAG}_$arg" "$arg" --steps 4 --warmup 1 --no-f32-pass --no-queued || exit 1; fi ;;
    levels)
        bash tools/gpu_level_pmc.sh "${arg}_$TAG" "$arg" > /dev/null || exit 1
        head -24 "$O/levels_${arg}_$TAG.txt" ;;
    bench)
        OUHIP_TUNE_CACHE="$O/tune_${TAG}_$arg.json" bench "$O/bench_${TAG}_config_$arg" 600 --config "$arg" || exit 1 ;;
    benchpmc)   # the PMC passes first, so the bench line carries its own library's traffic
        if [ "$arg" = c2 ]; then bash tools/gpu_profile.sh "${TAG}_pmc" c2 > /dev/null || exit 1
        else bash tools/gpu_profile.sh "${TAG}_pmc_$arg" "$arg" --steps 4 --warmup 1 --no-f32-pass --no-queued \
            > /dev/null || exit 1; fi
        pt="${TAG}_pmc$([ "$arg" = c2 ] || echo "_$arg")"   # the profile's tag: same tiles (its tuning cache)
        OUHIP_TUNE_CACHE="$O/tune_$pt.json" bench "$O/bench_${TAG}_config_$arg" 600 --config "$arg" \
            --traffic-json "$O/pmc_$pt.json" || exit 1 ;;
    shards)
        for b in 16 8 4; do
            OUHIP_TUNE_CACHE="$O/tune_${TAG}_c4.json" bench "$O/bench_${TAG}_c4_b$b" 300 --config c4 --batch $b \
                --steps 4 --warmup 1 --no-f32-pass --no-cpu-baseline --traffic-json "" || exit 1
        done ;;
    c4u)   # C4 on the undamped weights, quoting the traffic of its own PMC passes
        BENCH_EXTRA=--undamped bash tools/gpu_profile.sh "${TAG}_pmc_c4u" c4 --steps 3 --warmup 2 --no-f32-pass \
            --no-queued > /dev/null || exit 1
        OUHIP_TUNE_CACHE="$O/tune_${TAG}_pmc_c4u.json" bench "$O/bench_${TAG}_config_c4_undamped" 900 --config c4 \
            --undamped --steps 3 --warmup 2 --no-f32-pass --no-cpu-baseline \
            --traffic-json "$O/pmc_${TAG}_pmc_c4u.json" || exit 1 ;;
    critical)
        OUHIP_TUNE_CACHE="$O/tune_${TAG}_c2.json" timeout -k 10 300 python3 tools/critical_path.py --config c2 --reps 3 \
            --ops --out "$O/cp_$TAG.json" > "$O/cp_$TAG.txt" 2>&1 || { tail -20 "$O/cp_$TAG.txt"; exit 1; }
        grep -v "ou tune\|amdgpu" "$O/cp_$TAG.txt" | grep -B2 -A1 "first step" ;;
    ab)
        var=${arg%%=*}; val=${arg#*=}; base=0
        [[ "$val" == *,* ]] && { base=${val%%,*}; val=${val#*,}; }
        i=0
        for v in "$base" "$val" "$base" "$val"; do
            i=$((i + 1))
            ( export "$var=$v" OUHIP_TUNE_CACHE="$O/tune_${TAG}_c2.json"
              bench "$O/ab_${TAG}_${var}_${v}_$i" 200 --steps 20 --warmup 3 --no-cpu-baseline --no-f32-pass \
                  --no-queued --traffic-json "" ) || exit 1
        done ;;
    ablib)   # C2 bench: the in-tree library vs open_universe_amd/variants/libouhip_ARG.so, alternating
        for i in 1 2 3; do
            for lib in main "$arg"; do
                ( [ "$lib" = main ] || export OUHIP_LIB="$ROOT/open_universe_amd/variants/libouhip_$lib.so"
                  export OUHIP_TUNE_CACHE="$O/tune_${TAG}_$lib.json"
                  bench "$O/ab_${TAG}_${lib}_$i" 200 --steps 20 --warmup 3 --no-cpu-baseline --no-f32-pass \
                      --no-queued --traffic-json "" ) || exit 1
            done
        done ;;
    convsplit)   # tools/conv_bench.py --split on the deep-level layers (split-image kernel vs the best tile)
        timeout -k 10 300 python3 tools/conv_bench.py --layer ${arg:-L4k3,L4k5,L3k3,L3k5,GI,U3,U2,D3,D2} --reps 20 \
            --split > "$O/cbs_$TAG.txt" 2>&1 || { tail -20 "$O/cbs_$TAG.txt"; exit 1; }
        grep -v amdgpu "$O/cbs_$TAG.txt" | cut -c1-200 ;;
    convsplitlib)   # convsplit (k3 layers) with the in-tree library, then each variant of ARG (comma list)
        for lib in main ${arg//,/ }; do
            ( [ "$lib" = main ] || export OUHIP_LIB="$ROOT/open_universe_amd/variants/libouhip_$lib.so"
              st=""; [ "$lib" = stamps ] && st="--sstamps"
              timeout -k 10 300 python3 tools/conv_bench.py --layer L4k3,L3k3,U3,U2,D3,D2 --reps 20 --split $st \
                  > "$O/cbs_${TAG}_$lib.txt" 2>&1 ) || { tail -20 "$O/cbs_${TAG}_$lib.txt"; exit 1; }
            echo "## $lib"; grep -v amdgpu "$O/cbs_${TAG}_$lib.txt" | grep -v "^L\|^U\|^D\|^G" | cut -c1-200
        done ;;
    fir)   # tools/fir_bench.py: folded vs FIR-applied rate-change convs at config ARG (c4: FIR form only)
        fo=1; [ "${arg:-c4}" = c4 ] && fo=0
        timeout -k 10 400 python3 tools/fir_bench.py --config "${arg:-c4}" --folded $fo > "$O/fir_${TAG}_${arg:-c4}.txt" 2>&1 \
            || { tail -20 "$O/fir_${TAG}_${arg:-c4}.txt"; exit 1; }
        grep -v "ou tune\|amdgpu" "$O/fir_${TAG}_${arg:-c4}.txt" ;;
    firtile)   # one FIR-kernel layer on each of a list of tiles: ARG = CFG/LAYER/T1,T2,..
        IFS=/ read -r cfg lay tils <<< "$arg"
        for til in ${tils//,/ }; do
            timeout -k 10 120 python3 tools/fir_bench.py --config "$cfg" --only "$lay" --tile "$til" --reps 20 \
                2>&1 | grep "FIR tile" | tee -a "$O/firtile_${TAG}_${lay}.txt"
        done ;;
    sqconv|sqblock)   # SQ counters: sqconv:LAYER/TILE (tools/conv_bench.py), sqblock:LEVEL (PP24 block, B 32)
        if [ "$name" = sqconv ]; then
            IFS=/ read -r lay til <<< "$arg"; k=conv_kernel; out="$O/sqconv_${TAG}_$lay"
            cmd=(python3 "$ROOT/tools/conv_bench.py" --layer "$lay" --tile "$til" --reps 10)
        else
            k=block_kernel; out="$O/sqblock_${TAG}_L$arg"
            cmd=(python3 "$ROOT/tools/block_bench.py" --family pp24 --batch 32 --levels "$arg" --fused-only --reps 10)
        fi
        ( cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
              SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
              -d "${out}_a" -o pmc -- "${cmd[@]}" > "${out}_a.txt" 2>&1 ) || { tail -20 "${out}_a.txt"; exit 1; }
        ( cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
              SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv \
              -d "${out}_b" -o pmc -- "${cmd[@]}" > "${out}_b.txt" 2>&1 ) || { tail -20 "${out}_b.txt"; exit 1; }
        { grep -v amdgpu "${out}_a.txt" | tail -2
          python3 tools/pmc_avg.py "$(find "${out}_a" -name '*counter_collection.csv' | head -n1)" $k
          python3 tools/pmc_avg.py "$(find "${out}_b" -name '*counter_collection.csv' | head -n1)" $k; } > "$out.txt"
        cat "$out.txt" ;;
    sqfir)   # SQ counters of one FIR-kernel layer on a fixed tile: ARG = CFG/LAYER/TILE (e.g. c4/up0_r2/0x20000)
        IFS=/ read -r cfg lay til <<< "$arg"
        out="$O/sqfir_${TAG}_${lay}"
        ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
              SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
              -d "${out}_a" -o pmc -- python3 "$ROOT/tools/fir_bench.py" --config "$cfg" --only "$lay" --tile "$til" \
              --reps 10 > "${out}_a.txt" 2>&1 ) || { tail -20 "${out}_a.txt"; exit 1; }
        ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
              SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv \
              -d "${out}_b" -o pmc -- python3 "$ROOT/tools/fir_bench.py" --config "$cfg" --only "$lay" --tile "$til" \
              --reps 10 > "${out}_b.txt" 2>&1 ) || { tail -20 "${out}_b.txt"; exit 1; }
        k=conv_fdkernel; [[ "$lay" == up* ]] && k=conv_fukernel
        { grep -v amdgpu "${out}_a.txt" | tail -1
          python3 tools/pmc_avg.py "$(find "${out}_a" -name '*counter_collection.csv' | head -n1)" $k
          python3 tools/pmc_avg.py "$(find "${out}_b" -name '*counter_collection.csv' | head -n1)" $k; } > "$out.txt"
        cat "$out.txt" ;;
    convlib)   # tools/conv_bench.py on the deep-level layers: in-tree library vs variant ARG
        for lib in main "$arg"; do
            ( [ "$lib" = main ] || export OUHIP_LIB="$ROOT/open_universe_amd/variants/libouhip_$lib.so"
              timeout -k 10 300 python3 tools/conv_bench.py --layer L4k3,L4k5,L3k3,L3k5,GI,U3,U2 --reps 20 \
                  > "$O/cb_${TAG}_$lib.txt" 2>&1 ) || { tail -20 "$O/cb_${TAG}_$lib.txt"; exit 1; }
            echo "## $lib"; grep -v amdgpu "$O/cb_${TAG}_$lib.txt" | cut -c1-160
        done ;;
    *)
        echo "unknown step $step"; exit 2 ;;
    esac
done
