#!/usr/bin/env bash
# GPU: the given pytest selection (default: all -m gpu tests), one process,
# per-test timeout; output under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
LOG=gpurun_out/${LOGNAME_TAG:-pytest_gpu}.log
timeout -k 10 ${GPU_TEST_LIMIT:-900} python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    --durations=15 "${@:-tests}" > "$LOG" 2>&1
rc=$?
tail -40 "$LOG"
exit $rc
