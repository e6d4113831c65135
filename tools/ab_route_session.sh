#!/bin/bash
# Per-node routing A/B (round 4): SDMM_GUIDE_ROUTE=0/1, Morton key bits 10/8,
# Cornell K=128 and the K=512 product line; guide parity first.
L=sdmm-mitsuba_amd/lib/libsdmm_amd.so
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q -m gpu -x --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k guide \
    tests/test_gpu_wavefront.py tests/test_gpu_product.py tests/test_gpu_product_wavefront.py tests/test_gpu_li_oracle.py \
    tests/test_gpu_li.py > gpurun_out/abr_pytest.log 2>&1 || { tail -15 gpurun_out/abr_pytest.log; exit 1; }
tail -2 gpurun_out/abr_pytest.log
for cfg in "1 10" "0 10" "1 8"; do
  set -- $cfg
  echo "## route=$1 morton_bits=$2"
  SDMM_GUIDE_ROUTE=$1 SDMM_MORTON_BITS=$2 bash tools/corn_ab.sh "$L" 128 || exit 1
  SDMM_GUIDE_ROUTE=$1 SDMM_MORTON_BITS=$2 PRODUCT=1 bash tools/corn_ab.sh "$L" 512 || exit 1
done
