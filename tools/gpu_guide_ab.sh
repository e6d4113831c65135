#!/bin/bash
# Guide A/B on the GPU box: guide parity tests with the default library, then
# tools/guide_bench.py per library variant.  Usage: bash tools/gpu_guide_ab.sh TAG "variant ..."
TAG=$1; shift
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wavefront.py tests/test_gpu_product.py \
    tests/test_gpu_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/guide_tests_$TAG.log 2>&1
rc=$?; tail -3 $OUT/guide_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
for v in default $1; do
  if [ "$v" = default ]; then lib=""; else lib=sdmm-mitsuba_amd/build_ab/$v.so; fi
  GUIDE_CAP=${GUIDE_CAP:-} SDMM_AMD_LIB=$lib timeout -k 10 180 python tools/guide_bench.py > $OUT/guide_ab_${TAG}_$v.json 2> $OUT/guide_ab_${TAG}_$v.err
  rc=$?; echo "$v rc=$rc $(cat $OUT/guide_ab_${TAG}_$v.json)"
  [ $rc -eq 0 ] || { tail -5 $OUT/guide_ab_${TAG}_$v.err; exit $rc; }
done
