#!/bin/bash
# M-step phase breakdown: tools/em_phases.py (no RCCL) per library build
# (SDMM_MSTEP_STOP variants from tools/build_variant.sh).
# Usage: bash tools/mstep_ab.sh "lib1.so lib2.so ..."
OUT=gpurun_out; mkdir -p $OUT
for lib in $1; do
  SDMM_LIB_PATH=$PWD/$lib timeout -k 10 150 python tools/em_phases.py --no-rccl --reps 30 > $OUT/mab.log 2> $OUT/mab.err \
      || { tail -5 $OUT/mab.err; exit 1; }
  echo "$lib $(python3 -c "
import json
for l in open('$OUT/mab.log'):
    d = json.loads(l); print('w%d mstep %.1f us stats %.1f em %.1f |' % (d['world'], d['mstep_us'], d['estep_stats_us'], d['em_step_us']), end=' ')
")"
done
