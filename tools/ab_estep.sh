#!/bin/bash
# E-step A/B session on one box: the default build and the variants named on
# the command line (sdmm-mitsuba_amd/build_ab/NAME.so, tools/build_variant.sh),
# interleaved ROUNDS times; per process 100 event-timed launches
# (tools/resp_diag.py).  Usage: bash tools/ab_estep.sh TAG ROUNDS variant...
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/ab_$TAG.log
mkdir -p gpurun_out; : > "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for v in base "$@"; do
    if [ "$v" = base ]; then lib=""; else lib="sdmm-mitsuba_amd/build_ab/$v.so"; fi
    echo -n "$v " >> "$OUT"
    SDMM_LIB_PATH=${lib:-sdmm-mitsuba_amd/lib/libsdmm_amd.so} RESP_REPS=100 timeout -k 10 120 python tools/resp_diag.py >> "$OUT" 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc" >> "$OUT"; exit $rc; }
  done
done
python3 - "$OUT" <<'PY'
import json, sys, collections, statistics
d = collections.defaultdict(list)
h = collections.defaultdict(set)
for line in open(sys.argv[1]):
    name, js = line.split(" ", 1)
    r = json.loads(js)
    d[name].append(statistics.median(r["us"][60:]))
    h[name].add(r.get("sha256_16"))
for k, v in d.items():
    print(k, [round(x, 1) for x in v], "median", round(statistics.median(v), 1), "output", sorted(h[k]))
PY
