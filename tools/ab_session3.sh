#!/bin/bash
# Round-4 session 3: per-launch times of the split E-step configurations
# (variant 0: 8 waves at 2/SIMD; 2: 12 at 3), a rocprofv3 kernel trace of the
# variant-0 run (grid, LDS, VGPRs per dispatch), PAIR2 A/B.
B=sdmm-mitsuba_amd/build_ab; L=sdmm-mitsuba_amd/lib/libsdmm_amd.so
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out
for v in 0 2 0; do
  SDMM_RESP_VARIANT=$v timeout -k 10 120 python tools/resp_diag.py || exit 1
done
cd /tmp && SDMM_RESP_VARIANT=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_diag0 -o run \
    --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/resp_diag.py > $OUT/prof_diag0.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
SDMM_LIB_PATH=$PWD/$B/pr2.so SDMM_RESP_VARIANT=0 timeout -k 10 120 python tools/resp_diag.py || exit 1
SDMM_LIB_PATH=$PWD/$B/pr2n.so SDMM_RESP_VARIANT=0 timeout -k 10 120 python tools/resp_diag.py || exit 1
SDMM_LIB_PATH=$PWD/$B/lrn.so SDMM_RESP_VARIANT=0 timeout -k 10 120 python tools/resp_diag.py || exit 1
