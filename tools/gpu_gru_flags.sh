#!/usr/bin/env bash
# GPU: GRU recurrence variants (GRU_FLAGS list) at the score shape, then the
# chunked / unchunked kernel timelines.  Outputs under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
GRU_FLAGS=${GRU_FLAGS:-1,257,513,1} timeout -k 10 200 python -u tools/gru_bench.py > $O/grub_flags.log 2>&1 || exit $?
[ "${TIMELINE:-0}" = 1 ] || exit 0
cd /tmp
for m in 1 0; do
  OUHIP_CHUNK=$m timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl_$m -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-f32-pass --no-queued > $O/tl_$m.json 2> $O/tl_$m.err || exit $?
done
python3 $GRAFT_REPO_ROOT/tools/trace_timeline.py $(find $O/tl_1 -name "*kernel_trace.csv" | head -n1) --gru-per-enhance 26 > $O/tl_chunk.txt
python3 $GRAFT_REPO_ROOT/tools/trace_timeline.py $(find $O/tl_0 -name "*kernel_trace.csv" | head -n1) --gru-per-enhance 10 > $O/tl_nochunk.txt
