#!/bin/bash
# Round-4 session 5 (after the coefficient-image origin fix): per-launch
# times of the split E-step configurations, two processes each, and a golden
# responsibility check of every build first.
B=sdmm-mitsuba_amd/build_ab; L=sdmm-mitsuba_amd/lib/libsdmm_amd.so
export TMPDIR=/tmp
for lib in $L $B/regrows.so $B/pf2.so $B/pf4.so; do
  SDMM_LIB_PATH=$PWD/$lib timeout -k 10 120 python -m pytest -q -m gpu tests/test_gpu_golden.py > gpurun_out/ab5_golden.log 2>&1 \
    || { echo "golden failed: $lib"; tail -5 gpurun_out/ab5_golden.log; exit 1; }
done
echo "golden ok"
run() { SDMM_LIB_PATH=$PWD/$1 SDMM_RESP_VARIANT=$2 timeout -k 10 120 python tools/resp_diag.py | \
        python3 -c "import json,sys,statistics as s; d=json.loads(sys.stdin.read()); print('$1 v$2', d['kernel'], 'median', s.median(d['us']), 'min', min(d['us']), 'max', max(d['us']))"; }
for i in 1 2; do
  run $L 0 || exit 1; run $L 3 || exit 1; run $B/regrows.so 3 || exit 1; run $B/regrows.so 0 || exit 1
  run $B/pf2.so 0 || exit 1; run $B/pf4.so 0 || exit 1; run $B/pf2.so 3 || exit 1
done
run $B/storeonly.so 0 || exit 1
