#!/bin/bash
# A/B of the headline responsibility E-step kernels: SDMM_RESP_KERNEL x
# SDMM_RESP_VARIANT pairs ("kernel:variant"), each a short bench.py run.
# Usage: bash tools/gpu_split_ab.sh "tile:4 split:0 split:1"
OUT=gpurun_out; mkdir -p $OUT
for kv in $1; do
  k=${kv%%:*}; v=${kv##*:}
  SDMM_RESP_KERNEL=$k SDMM_RESP_VARIANT=$v timeout -k 10 120 python bench.py --no-cpu --no-extra --steps 30 --warmup 10 \
      > $OUT/sab.json 2> $OUT/sab.err || { tail -5 $OUT/sab.err; exit 1; }
  echo "$kv $(python3 -c "import json;d=json.load(open('$OUT/sab.json'));r=d['roofline'];print(r['kernel'], round(r['kernel_us'],1), 'us frac', round(r['frac'],3), 'ms/step', round(d['ms_per_step'],4))")"
done
