#!/bin/bash
# Round-4 A/B session 2: guide two-pass candidate selection on the Cornell
# renders (K=128 plain, K=512 product), the split E-step repeatability check,
# the M-step phase breakdown.  Each step has its own time limit.
B=sdmm-mitsuba_amd/build_ab; L=sdmm-mitsuba_amd/lib/libsdmm_amd.so
export TMPDIR=/tmp
bash tools/gpu_resp_ab.sh "$L $L $B/lr2.so" 0 || exit 1
bash tools/gpu_resp_ab.sh "$B/lrn.so" 2 || exit 1
bash tools/corn_ab.sh "$L $B/twopass.so" 128 || exit 1
PRODUCT=1 bash tools/corn_ab.sh "$L $B/twopass.so" 512 || exit 1
bash tools/mstep_ab.sh "$B/mstop1.so $B/mstop2.so $B/mstop3.so $B/mstop4.so $L" || exit 1
