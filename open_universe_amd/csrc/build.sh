#!/usr/bin/env bash
# Build libouhip.so for gfx950 (MI355X).  Cross-compiles without a GPU.
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
OUT="${1:-$HERE/../libouhip.so}"
ARCH="${OUHIP_ARCH:-gfx950}"
OBJDIR="$HERE/build${OUHIP_BUILD_TAG:-}"
mkdir -p "$OBJDIR"
SRCS="ou_conv.hip ou_gru.hip ou_misc.hip ou_program.hip ou_audio.hip"
pids=()
for s in $SRCS; do
  /opt/rocm/bin/hipcc --offload-arch="$ARCH" -O3 -fPIC -std=c++17 -Wall -Wno-unused-function ${OUHIP_CFLAGS:-} \
      -c "$HERE/$s" -o "$OBJDIR/${s%.hip}.o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc --offload-arch="$ARCH" -shared -fPIC -o "$OUT" "$OBJDIR"/*.o
echo "built $OUT"
