#!/bin/bash
# K=512 Cornell product guided pass per SDMM_PRODUCT_ROUTE_PAIRS value
# (candidate queries with more kept x lobe pairs go to the one-wave path).
# Usage: bash tools/ab_route_cornell.sh T1 T2 ...   ("default": unset)
OUT=gpurun_out/ab_route_cornell.log
mkdir -p gpurun_out; : > "$OUT"
for t in "$@"; do
  if [ "$t" = default ]; then unset SDMM_PRODUCT_ROUTE_PAIRS; else export SDMM_PRODUCT_ROUTE_PAIRS=$t; fi
  timeout -k 10 300 python tools/cornell_bench.py --K 512 --modes 0 --product > gpurun_out/abr_run.log 2>&1 || exit 1
  python3 - "$t" gpurun_out/abr_run.log >> "$OUT" <<'PY'
import json, sys, statistics
its = [json.loads(l) for l in open(sys.argv[2]) if l.startswith('{"ms"')]
g = [x["ms"] for x in its if not x["train"]]
t = [x["ms"] for x in its if x["train"]]
print("route", sys.argv[1], json.dumps({"guided_ms_median": statistics.median(g), "train_ms": t}))
PY
done
cat "$OUT"
