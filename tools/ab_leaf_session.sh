#!/bin/bash
# Leaf-major coherent order A/B (round 4): SDMM_LEAF_ORDER=1 (default) / 0.
L=sdmm-mitsuba_amd/lib/libsdmm_amd.so
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q -m gpu -x --timeout 120 --timeout-method thread tests/test_gpu_wavefront.py \
    tests/test_gpu_product_wavefront.py tests/test_gpu_li_oracle.py tests/test_gpu_li.py > gpurun_out/abl_pytest.log 2>&1 \
    || { tail -15 gpurun_out/abl_pytest.log; exit 1; }
tail -1 gpurun_out/abl_pytest.log
for o in 1 0; do
  echo "## leaf_order=$o"
  SDMM_LEAF_ORDER=$o bash tools/corn_ab.sh "$L" 16 || exit 1
  SDMM_LEAF_ORDER=$o bash tools/corn_ab.sh "$L" 128 || exit 1
  SDMM_LEAF_ORDER=$o PRODUCT=1 bash tools/corn_ab.sh "$L" 512 || exit 1
done
