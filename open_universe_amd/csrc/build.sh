#!/usr/bin/env bash
# Build libouhip.so for gfx950 (MI355X).  Cross-compiles without a GPU.
# ou_conv.hip is compiled as one unit per tap count (OU_CONV_SPLIT_KT) plus the
# C ABI unit (OU_CONV_SPLIT_MAIN), so its many kernel instantiations build in
# parallel.  OUHIP_CFLAGS containing OU_CONV_STAMPS builds it as one unit.
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
OUT="${1:-$HERE/../libouhip.so}"
ARCH="${OUHIP_ARCH:-gfx950}"
OBJDIR="$HERE/build${OUHIP_BUILD_TAG:-}"
mkdir -p "$OBJDIR"
# OUHIP_INCREMENTAL=1 (development): keep objects newer than their source and
# the shared headers; the default rebuilds everything
[ "${OUHIP_INCREMENTAL:-0}" = 1 ] || rm -f "$OBJDIR"/*.o
CFLAGS=(--offload-arch="$ARCH" -O3 -fPIC -std=c++17 -Wall -Wno-unused-function)
pids=()
cc() {   # cc <src> <obj> [extra flags...]
  local src="$1" obj="$2"; shift 2
  if [ -f "$OBJDIR/$obj" ] && [ "$OBJDIR/$obj" -nt "$HERE/$src" ] && [ "$OBJDIR/$obj" -nt "$HERE/ou_common.h" ] \
     && [ "$OBJDIR/$obj" -nt "$HERE/../../include/ouhip.h" ]; then return 0; fi
  /opt/rocm/bin/hipcc "${CFLAGS[@]}" ${OUHIP_CFLAGS:-} "$@" -c "$HERE/$src" -o "$OBJDIR/$obj" &
  pids+=($!)
}
for s in ou_gru.hip ou_misc.hip ou_program.hip ou_audio.hip ou_block.hip; do
  cc "$s" "${s%.hip}.o"
done
cc ou_flac.cpp ou_flac.o   # host-only (FLAC input decoding for the CLI)
if [[ "${OUHIP_CFLAGS:-}" == *OU_CONV_STAMPS* ]]; then
  cc ou_conv.hip ou_conv.o
else
  cc ou_conv.hip ou_conv_main.o -DOU_CONV_SPLIT_MAIN
  for k in 1 3 4 5; do
    cc ou_conv.hip "ou_conv_k$k.o" -DOU_CONV_SPLIT_KT=$k
  done
  for r in 2 3 4 5 8; do   # the FIR-applied rate-change kernels, one unit per rate
    cc ou_conv.hip "ou_conv_fir$r.o" -DOU_CONV_SPLIT_FIR=$r
  done
fi
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=1; done
[ "$rc" -eq 0 ] || { echo "build failed" >&2; exit 1; }
/opt/rocm/bin/hipcc --offload-arch="$ARCH" -shared -fPIC -o "$OUT" "$OBJDIR"/*.o
echo "built $OUT"
