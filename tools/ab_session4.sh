#!/bin/bash
# Round-4 session 4: split E-step with round-robin tiles (per-launch times,
# several processes per configuration), the M-step finish rewrite.
B=sdmm-mitsuba_amd/build_ab; L=sdmm-mitsuba_amd/lib/libsdmm_amd.so
export TMPDIR=/tmp
run() { SDMM_LIB_PATH=$PWD/$1 SDMM_RESP_VARIANT=$2 timeout -k 10 120 python tools/resp_diag.py | \
        python3 -c "import json,sys,statistics as s; d=json.loads(sys.stdin.read()); print('$1 v$2', d['kernel'], 'median', s.median(d['us']), 'min', min(d['us']), 'max', max(d['us']))"; }
for i in 1 2; do run $L 0 || exit 1; run $L 2 || exit 1; done
run $B/lrn.so 2 || exit 1; run $B/lrn.so 0 || exit 1; run $B/lr2.so 0 || exit 1
run $B/pr2.so 0 || exit 1; run $B/pr2n.so 0 || exit 1; run $B/scalar.so 0 || exit 1; run $B/storeonly.so 0 || exit 1
run $L 0 || exit 1
bash tools/mstep_ab.sh "$B/finwave.so $L" || exit 1
