#!/usr/bin/env bash
# GPU: bench (fills the tuning cache) -> rocprofv3 kernel-trace/stats of the
# bench -> two PMC passes (FETCH_SIZE, WRITE_SIZE) -> per-kernel traffic.
# Usage: tools/gpu_profile.sh TAG [CONFIG [bench args...]]   (outputs under gpurun_out/*_TAG)
#   CONFIG: bench.py --config (default c2); the remaining args go to the first
#   (timed) bench run, e.g. "--steps 5 --warmup 2 --no-f32-pass" for c4;
#   BENCH_EXTRA (env): arguments for every bench run of the script (e.g. --undamped)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-run}
CFG=${2:-c2}
shift 2 2>/dev/null || shift $#
FIRST=("$@")
[ ${#FIRST[@]} -gt 0 ] || FIRST=(--steps 20 --warmup 3)
O="$ROOT/gpurun_out"
mkdir -p "$O"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
export OUHIP_TUNE_CACHE="$O/tune_$TAG.json"
B="$ROOT/bench.py"
read -r -a EXTRA <<< "${BENCH_EXTRA:-}"
timeout -k 10 600 python3 "$B" --config "$CFG" "${EXTRA[@]}" "${FIRST[@]}" --dump-ops "$O/ops_$TAG.json" \
    > "$O/bench_$TAG.json" 2> "$O/bench_$TAG.err" &&
cd /tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_$TAG" -o kt -- \
    python3 "$B" --config "$CFG" "${EXTRA[@]}" --steps 5 --warmup 1 --no-cpu-baseline --no-profile --no-f32-pass --no-queued > "$O/kt_bench_$TAG.json" 2> "$O/kt_$TAG.err" &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmcf_$TAG" -o pmc -- \
    python3 "$B" --config "$CFG" "${EXTRA[@]}" --steps 1 --warmup 1 --no-cpu-baseline --no-profile --no-f32-pass --no-queued > /dev/null 2> "$O/pmcf_$TAG.err" &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmcw_$TAG" -o pmc -- \
    python3 "$B" --config "$CFG" "${EXTRA[@]}" --steps 1 --warmup 1 --no-cpu-baseline --no-profile --no-f32-pass --no-queued > /dev/null 2> "$O/pmcw_$TAG.err" &&
python3 "$ROOT/tools/pmc_summary.py" --tag "$TAG" --config "$CFG" --enhances 2 --out "$O/pmc_$TAG.json" \
    --lib "$ROOT/open_universe_amd/libouhip.so" \
    "$(find "$O/pmcf_$TAG" -name '*counter_collection.csv' | head -n1)" \
    "$(find "$O/pmcw_$TAG" -name '*counter_collection.csv' | head -n1)" > /dev/null
rc=$?
[ "$rc" -eq 0 ] && python3 "$ROOT/tools/trace_gaps.py" "$(find "$O/kt_$TAG" -name '*kernel_trace.csv' | head -n1)" \
    > "$O/trace_gaps_$TAG.txt"
cat "$O/bench_$TAG.json"
find "$O/kt_$TAG" -name '*kernel_stats.csv' -exec head -n 12 {} \;
exit $rc
