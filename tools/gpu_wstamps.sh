#!/usr/bin/env bash
# Warp-specialised conv phase stamps on a few layers (diagnostic library).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 OUHIP_LIB=open_universe_amd/libouhip_stamps.so
for L in L0k3 L1k3 L4k3; do
  for T in ${TILES:-1024 1027 1035}; do
    timeout -k 10 120 python tools/conv_bench.py --layer $L --tile $T --reps 3 --wstamps || exit 1
  done
done > gpurun_out/wstamps.log 2>&1
rc=$?
cat gpurun_out/wstamps.log
exit $rc
