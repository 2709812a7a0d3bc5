#!/bin/bash
# Timing-only variant libraries (wrong results) for A/B runs through AST_HIP_LIB:
#   bash scripts/build_variants.sh NAME "-DFLAG=1 ..." [source.hip]
# rebuilds SOURCE (default mb_ed4.hip; a csrc file name, or a path to another version of one, e.g.
# build_var/src_old/conv3x3_igemm.hip from git show) with the flags and links it with the other
# in-tree objects into build_var/libast_hip_NAME.so. Run `make -C arbitrarystyletransfer_amd/csrc` first.
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
NAME="$1"; FLAGS="$2"; SRCP="${3:-mb_ed4.hip}"
C="$ROOT/arbitrarystyletransfer_amd/csrc"; OUT="$ROOT/build_var"; mkdir -p "$OUT/$NAME"
case "$SRCP" in */*) ;; *) SRCP="$C/$SRCP" ;; esac
SRC="$(basename "$SRCP")"
extra=""; [ "$SRC" = mb_ed4.hip ] && extra="-fno-slp-vectorize"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$ROOT/include" -I"$C" $extra \
  -Xclang -target-feature -Xclang -packed-fp32-ops $FLAGS -c "$SRCP" -o "$OUT/$NAME/${SRC%.hip}.o" 2>&1 \
  | { grep -v "not a recognized feature" || true; }
objs=""
for o in "$C"/build/*.o; do
  b=$(basename "$o"); [ "$b" = "${SRC%.hip}.o" ] && o="$OUT/$NAME/$b"; [ "$b" = torch_ops.o ] && continue; objs="$objs $o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libast_hip_$NAME.so" $objs
echo "$OUT/libast_hip_$NAME.so"
