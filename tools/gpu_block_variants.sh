#!/usr/bin/env bash
# GPU: tools/block_bench.py with the in-tree library and each variant build
# of ou_block.hip (open_universe_amd/variants/libouhip_NAME.so).
# Usage: tools/gpu_block_variants.sh TAG NAME...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
export PYTHONUNBUFFERED=1
TAG=$1; shift
out=$O/block_variants_$TAG.txt
echo "== base" > $out
timeout -k 10 200 python -u tools/block_bench.py --levels 0,1,2 2>/dev/null | grep '^{' >> $out || exit $?
for v in "$@"; do
  echo "== $v" >> $out
  OUHIP_LIB=$PWD/open_universe_amd/variants/libouhip_$v.so timeout -k 10 200 python -u tools/block_bench.py --levels 0,1,2 2>/dev/null | grep '^{' >> $out || exit $?
done
cat $out
