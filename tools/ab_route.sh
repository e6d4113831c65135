#!/bin/bash
# Product routing A/B (SDMM_PRODUCT_ROUTE_PAIRS: candidate-served product
# queries with more kept x lobe pairs go to the one-wave path): the Kitchen
# product (tools/product_bench.py, capacity 40) and the K=512 Cornell product
# passes (diffuse and glossy), per threshold.  Usage: bash tools/ab_route.sh T1 T2 ...
OUT=gpurun_out/ab_route.log
mkdir -p gpurun_out; : > "$OUT"
for t in "$@"; do
  if [ "$t" = off ]; then unset SDMM_PRODUCT_ROUTE_PAIRS; else export SDMM_PRODUCT_ROUTE_PAIRS=$t; fi
  echo -n "route=$t kitchen: " >> "$OUT"
  timeout -k 10 200 python tools/product_bench.py --caps 40 --reps 5 2>/dev/null | tr '\n' ' ' >> "$OUT" || exit 1
  echo >> "$OUT"
done
cat "$OUT"
