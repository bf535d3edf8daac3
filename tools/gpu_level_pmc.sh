#!/usr/bin/env bash
# GPU: per-op conv-stack table (tools/level_pmc.py): one timing run, then one
# rocprofv3 pass per counter.  Usage: tools/gpu_level_pmc.sh TAG CONFIG [run args]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=$1; CFG=$2; shift 2
O="$ROOT/gpurun_out"; mkdir -p "$O"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
export OUHIP_TUNE_CACHE="$O/tune_$TAG.json"
P="$ROOT/tools/level_pmc.py"
timeout -k 10 300 python3 "$P" run --config "$CFG" "$@" --out "$O/lvops_$TAG.json" > "$O/lv_$TAG.log" 2>&1 &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/lvf_$TAG" -o pmc -- \
    python3 "$P" run --config "$CFG" "$@" --out "$O/lvops_f_$TAG.json" >> "$O/lv_$TAG.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/lvw_$TAG" -o pmc -- \
    python3 "$P" run --config "$CFG" "$@" --out "$O/lvops_w_$TAG.json" >> "$O/lv_$TAG.log" 2>&1 &&
python3 "$P" analyze "$O/lvops_$TAG.json" \
    "$(find "$O/lvf_$TAG" -name '*counter_collection.csv' | head -n1)" \
    "$(find "$O/lvw_$TAG" -name '*counter_collection.csv' | head -n1)" --out "$O/levels_$TAG.json" \
    > "$O/levels_$TAG.txt"
rc=$?
cat "$O/levels_$TAG.txt"
exit $rc
