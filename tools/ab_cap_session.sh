#!/bin/bash
# Candidate capacity A/B (round 4): default 40 vs 48 / 56 (top LCAP tier).
B=sdmm-mitsuba_amd/build_ab; L=sdmm-mitsuba_amd/lib/libsdmm_amd.so
export TMPDIR=/tmp
for lib in $B/c48.so $B/c56.so; do
  SDMM_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u -m pytest -q -m gpu -x --timeout 120 --timeout-method thread \
      tests/test_gpu_wavefront.py tests/test_gpu_product_wavefront.py -k "not -64] and not -64-" > gpurun_out/abc_pytest.log 2>&1 \
      || { echo "parity failed: $lib"; tail -15 gpurun_out/abc_pytest.log; exit 1; }
done
echo parity ok
bash tools/corn_ab.sh "$L $B/c48.so $B/c56.so" 128 || exit 1
PRODUCT=1 bash tools/corn_ab.sh "$L $B/c48.so $B/c56.so" 512 || exit 1
