#!/bin/bash
# Morton-order threshold A/B (round 4): SDMM_TREE_ORDER_MIN over the Cornell
# K=16 and K=128 lines.
L=sdmm-mitsuba_amd/lib/libsdmm_amd.so
export TMPDIR=/tmp
for m in 16384 65536 262144 1000000000; do
  echo "## order_min=$m"
  SDMM_TREE_ORDER_MIN=$m bash tools/corn_ab.sh "$L" 16 || exit 1
  SDMM_TREE_ORDER_MIN=$m bash tools/corn_ab.sh "$L" 128 || exit 1
done
