#!/bin/bash
# Full-K group fallback A/B (round 4): 4-lane groups (default) vs 16-lane.
B=sdmm-mitsuba_amd/build_ab; L=sdmm-mitsuba_amd/lib/libsdmm_amd.so
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q -m gpu -x --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k guide \
    tests/test_gpu_wavefront.py tests/test_gpu_li_oracle.py > gpurun_out/abgr_pytest.log 2>&1 \
    || { tail -15 gpurun_out/abgr_pytest.log; exit 1; }
tail -2 gpurun_out/abgr_pytest.log
bash tools/corn_ab.sh "${LIBS:-$L $B/gg16.so}" 128 || exit 1
