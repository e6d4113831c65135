#!/bin/bash
# K=128 Cornell guided-pass A/B: the default build and the variants named
# (sdmm-mitsuba_amd/build_ab/NAME.so), interleaved ROUNDS times.
# Usage: bash tools/ab_k128.sh TAG ROUNDS variant...
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/abk_$TAG.log
mkdir -p gpurun_out; : > "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for v in base "$@"; do
    if [ "$v" = base ]; then lib=sdmm-mitsuba_amd/lib/libsdmm_amd.so; else lib="sdmm-mitsuba_amd/build_ab/$v.so"; fi
    SDMM_LIB_PATH=$lib timeout -k 10 300 python tools/cornell_bench.py --K 128 --modes 0 > gpurun_out/abk_run.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc" >> "$OUT"; cat gpurun_out/abk_run.log >> "$OUT"; exit $rc; }
    python3 - "$v" gpurun_out/abk_run.log >> "$OUT" <<'PY'
import json, sys, statistics
its = [json.loads(l) for l in open(sys.argv[2]) if l.startswith('{"ms"')]
g = [x["ms"] for x in its if not x["train"]]
t = [x["ms"] for x in its if x["train"]]
print(sys.argv[1], json.dumps({"guided_ms_median": statistics.median(g), "train_ms": t}))
PY
  done
done
cat "$OUT"
