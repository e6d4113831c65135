#!/bin/bash
# A/B of the responsibility kernels on the GPU box: headline bench line per
# (SDMM_RESP_KERNEL, SDMM_RESP_VARIANT).  Usage: bash tools/gpu_ab.sh TAG "kernel:variant ..."
TAG=$1; shift
OUT=gpurun_out; mkdir -p $OUT
for kv in $1; do
  k=${kv%%:*}; v=${kv##*:}
  SDMM_RESP_KERNEL=$k SDMM_RESP_VARIANT=$v timeout -k 10 120 python bench.py --no-cpu --no-extra --steps 20 --warmup 5 \
      > $OUT/ab_${TAG}_${k}_${v}.json 2> $OUT/ab_${TAG}_${k}_${v}.err
  rc=$?
  echo "$k:$v rc=$rc $(python3 -c "import json,sys;d=json.load(open('$OUT/ab_${TAG}_${k}_${v}.json'));r=d['roofline'];print(r['kernel'], round(r['kernel_us'],1), 'us frac', round(r['frac'],3))" 2>/dev/null)"
  [ $rc -eq 0 ] || exit $rc
done
