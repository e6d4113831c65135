#!/bin/bash
# Round-4 session 10: the default block loop without its scheduling fences.
B=sdmm-mitsuba_amd/build_ab; L=sdmm-mitsuba_amd/lib/libsdmm_amd.so
export TMPDIR=/tmp
run() { SDMM_LIB_PATH=$PWD/$1 SDMM_RESP_VARIANT=$2 timeout -k 10 120 python tools/resp_diag.py | \
        python3 -c "import json,sys,statistics as s; d=json.loads(sys.stdin.read()); print('$1 v$2', d['kernel'], 'median', s.median(d['us']), 'min', min(d['us']), 'max', max(d['us']))"; }
SDMM_LIB_PATH=$PWD/$B/nofence.so timeout -k 10 120 python -m pytest -q -m gpu tests/test_gpu_golden.py > gpurun_out/ab10_golden.log 2>&1 || { tail -5 gpurun_out/ab10_golden.log; exit 1; }
for i in 1 2 3; do run $L 0 || exit 1; run $B/nofence.so 0 || exit 1; done
