#!/bin/bash
# Stage costs of the one-wave full-K product path by difference: builds made
# with -DSDMM_PW_STOP=4/1/2/3 (tools/build_variant.sh stopN "-DSDMM_PW_STOP=N"
# csrc/guide.hip) return after the slot weights / the preparation / pass 1 /
# pass 2; each is timed on the Kitchen product workload (tools/product_bench.py,
# capacity 0: every query on the wave path; 40: the default).  Outputs of the
# stop builds are not the product's.  Usage (on the box): bash tools/product_stages.sh
set -e
OUT=gpurun_out/stages.log
mkdir -p gpurun_out; : > "$OUT"
for v in base stop4 stop1 stop2 stop3 base; do
  if [ $v = base ]; then lib=sdmm-mitsuba_amd/lib/libsdmm_amd.so; else lib=sdmm-mitsuba_amd/build_ab/$v.so; fi
  echo -n "$v " >> "$OUT"
  SDMM_LIB_PATH=$lib timeout -k 10 200 python tools/product_bench.py --caps 0,40 --reps 5 2>/dev/null | tr '\n' ' ' >> "$OUT"
  echo >> "$OUT"
done
cat "$OUT"
