#!/usr/bin/env bash
# One GPU session: smoke, then the GPU parity tests.  Each GPU step has its own
# time limit; steps are chained with && so nothing runs after a failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/smoke.log; tail -30 gpurun_out/pytest_gpu.log
exit $rc
