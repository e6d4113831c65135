#!/bin/bash
# A/B session on the GPU box (round 4): split E-step variants (variant 0:
# 8-wave workgroups at 2 waves/SIMD; 2: 12 waves at 3), then the EM phase
# breakdown.  Every step has its own time limit; a failure ends the session.
B=sdmm-mitsuba_amd/build_ab; L=sdmm-mitsuba_amd/lib/libsdmm_amd.so
export TMPDIR=/tmp
bash tools/gpu_resp_ab.sh "$L $B/scalar.so $B/pipe10.so $B/pipe18s.so $B/storeonly.so" 0 || exit 1
bash tools/gpu_resp_ab.sh "$B/lr2.so" 0 || exit 1
bash tools/gpu_resp_ab.sh "$B/lrn.so $B/lrns.so" 2 || exit 1
bash tools/gpu_resp_ab.sh "$L" 0 || exit 1
timeout -k 10 180 python tools/em_phases.py > gpurun_out/em_phases.log 2>&1; rc=$?
tail -4 gpurun_out/em_phases.log; exit $rc
