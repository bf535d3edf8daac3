set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$PWD/gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 200 python -u tools/gru_bench.py > $O/grub1.log 2>&1 || exit $?
cd /tmp
OUHIP_CHUNK=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl_chunk -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-f32-pass --no-queued > $O/tl_chunk.json 2> $O/tl_chunk.err || exit $?
OUHIP_CHUNK=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl_nochunk -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-f32-pass --no-queued > $O/tl_nochunk.json 2> $O/tl_nochunk.err || exit $?
