#!/bin/bash
# Guided-query A/B (round 4): the candidate-list builders and capacities.
# Parity of the default build first, then per build the Cornell K=128 line,
# the K=512 product line and the single-mixture guide microbenchmark.
B=sdmm-mitsuba_amd/build_ab; L=sdmm-mitsuba_amd/lib/libsdmm_amd.so
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q -m gpu -x --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k guide \
    tests/test_gpu_wavefront.py tests/test_gpu_product.py tests/test_gpu_product_wavefront.py tests/test_gpu_li_oracle.py \
    > gpurun_out/abg_pytest.log 2>&1 || { tail -15 gpurun_out/abg_pytest.log; exit 1; }
tail -2 gpurun_out/abg_pytest.log
LIBS=${LIBS:-"$L $B/gcap40.so $B/gold.so"}
bash tools/corn_ab.sh "$LIBS" 128 || exit 1
PRODUCT=1 bash tools/corn_ab.sh "$LIBS" 512 || exit 1
for lib in $LIBS; do
  SDMM_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/guide_bench.py > gpurun_out/abg_gb.json 2> gpurun_out/abg_gb.err \
      || { tail -5 gpurun_out/abg_gb.err; exit 1; }
  echo "$lib $(cat gpurun_out/abg_gb.json)"
done
