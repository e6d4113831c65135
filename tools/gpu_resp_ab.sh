#!/bin/bash
# A/B of the headline responsibility E-step: library builds (SDMM_LIB_PATH) x
# split variants (SDMM_RESP_VARIANT), each a short bench.py --no-extra run.
# Usage: bash tools/gpu_resp_ab.sh "lib1.so lib2.so" "0 1"
OUT=gpurun_out; mkdir -p $OUT
for lib in $1; do
  for v in $2; do
    SDMM_LIB_PATH=$PWD/$lib SDMM_RESP_VARIANT=$v timeout -k 10 120 python bench.py --no-cpu --no-extra --steps 30 --warmup 10 \
        > $OUT/rab.json 2> $OUT/rab.err || { tail -5 $OUT/rab.err; exit 1; }
    echo "$lib v$v $(python3 -c "import json;d=json.load(open('$OUT/rab.json'));r=d['roofline'];print(r['kernel'], round(r['kernel_us'],1), 'us frac', round(r['frac'],3))")"
  done
done
