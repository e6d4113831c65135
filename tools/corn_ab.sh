#!/bin/bash
# Cornell guided-render A/B over library builds (SDMM_LIB_PATH): per build the
# cornell_bench line at the given K (and --product if PRODUCT=1), summarised.
# Usage: bash tools/corn_ab.sh "lib1.so lib2.so" "128"
OUT=gpurun_out; mkdir -p $OUT
for lib in $1; do
  extra=""; [ "${PRODUCT:-0}" = 1 ] && extra="--product"
  SDMM_LIB_PATH=$PWD/$lib timeout -k 10 240 python tools/cornell_bench.py --K $2 --modes 0 $extra > $OUT/cab.log 2> $OUT/cab.err \
      || { tail -5 $OUT/cab.err; exit 1; }
  echo "== $lib"; python3 tools/corn_summary.py < $OUT/cab.log
done
