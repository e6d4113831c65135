#!/bin/bash
# Round-4 session 6: split E-step prologue cost -- the coefficient image
# build against a zero image (diagnostic), with and without the math.
B=sdmm-mitsuba_amd/build_ab; L=sdmm-mitsuba_amd/lib/libsdmm_amd.so
export TMPDIR=/tmp
run() { SDMM_LIB_PATH=$PWD/$1 SDMM_RESP_VARIANT=$2 timeout -k 10 120 python tools/resp_diag.py | \
        python3 -c "import json,sys,statistics as s; d=json.loads(sys.stdin.read()); print('$1 v$2', d['kernel'], 'median', s.median(d['us']), 'min', min(d['us']), 'max', max(d['us']))"; }
for i in 1 2; do
  run $L 0 || exit 1; run $B/noimg.so 0 || exit 1; run $B/so.so 0 || exit 1; run $B/soni.so 0 || exit 1
done
