#!/usr/bin/env bash
# GPU: run several steps in order, each under its own time limit, stopping at
# the first step that crashed, faulted, aborted or timed out (exit >= 124 or a
# signal); an ordinary failure (pytest rc 1, a bench error) is reported and
# the next step still runs.  Usage:
#   tools/gpu_chain.sh 'SECONDS:command' 'SECONDS:command' ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
worst=0
for step in "$@"; do
  secs="${step%%:*}"
  cmd="${step#*:}"
  echo "[chain] $(date +%T) start (${secs}s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd"
  rc=$?
  echo "[chain] $(date +%T) rc=$rc: $cmd"
  if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then
    echo "[chain] stopping: crash / abort / timeout"
    exit "$rc"
  fi
  [ "$rc" -gt "$worst" ] && worst=$rc
done
exit "$worst"
