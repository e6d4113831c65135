#!/bin/bash
# Build a variant of lib/libsdmm_amd.so for A/B runs: the listed sources are
# recompiled with extra flags, the other objects come from the regular build.
# Usage: bash tools/build_variant.sh NAME "EXTRA FLAGS" csrc/guide.hip [more sources]
set -e
NAME=$1; FLAGS=$2; shift 2
PKG=$(cd "$(dirname "$0")/../sdmm-mitsuba_amd" && pwd)
make -s -C "$PKG"
OUT=$PKG/build/ab/$NAME; mkdir -p "$OUT" "$PKG/build_ab"
HIPFLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function -Wno-unused-variable -munsafe-fp-atomics -fgpu-flush-denormals-to-zero"
OBJS=()
for o in "$PKG"/build/*.o; do
  src=csrc/$(basename "$o" .o)
  if printf '%s\n' "$@" | grep -qx "$src"; then
    EXTRA=""   # the Makefile's E-step rule: no SLP re-packing
    case "$src" in csrc/estep*.hip) EXTRA="-fno-slp-vectorize";; esac
    /opt/rocm/bin/hipcc $HIPFLAGS $EXTRA $FLAGS -x hip -c "$PKG/$src" -o "$OUT/$(basename "$o")"
    OBJS+=("$OUT/$(basename "$o")")
  else
    OBJS+=("$o")
  fi
done
/opt/rocm/bin/hipcc $HIPFLAGS -shared -o "$PKG/build_ab/$NAME.so" "${OBJS[@]}" -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "$PKG/build_ab/$NAME.so"
