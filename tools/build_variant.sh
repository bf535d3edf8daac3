#!/usr/bin/env bash
# Experiment builds: recompile ONE source of libouhip.so with extra flags and
# link it with the other objects of the last full build (csrc/build/) into
# open_universe_amd/variants/libouhip_NAME.so (gitignored; travels to the GPU
# box with the tree).  Select one at run time with OUHIP_LIB=<path>.
#   tools/build_variant.sh NAME SOURCE "FLAGS" [OBJECT]   e.g. ring10 ou_block.hip "-DOU_BLOCK_RING1=10"
# OBJECT: the build/ object the variant replaces (default SOURCE's), e.g. one
# tap-count unit of ou_conv.hip:  nb ou_conv.hip "-DOU_CONV_SPLIT_KT=3 -DX=0" ou_conv_k3.o
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
CS="$ROOT/open_universe_amd/csrc"
NAME="$1"; SRC="$2"; FLAGS="${3:-}"; OBJNAME="${4:-${SRC%.hip}.o}"
OUT="$ROOT/open_universe_amd/variants"
mkdir -p "$OUT" "$OUT/obj_$NAME"
OBJ="$OUT/obj_$NAME/$OBJNAME"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function $FLAGS -c "$CS/$SRC" -o "$OBJ"
objs=()
for o in "$CS"/build/*.o; do
  [ "$(basename "$o")" = "$(basename "$OBJ")" ] || objs+=("$o")
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libouhip_$NAME.so" "${objs[@]}" "$OBJ"
rm -rf "$OUT/obj_$NAME"
echo "built $OUT/libouhip_$NAME.so"
