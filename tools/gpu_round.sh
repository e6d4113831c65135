#!/bin/bash
# One GPU-box session: GPU tests, bench, rocprofv3 kernel-trace summary.
# Each GPU step has its own time limit; a fault / abort / timeout ends the
# script (only ordinary test failures, rc 1, let it continue).
# Usage (from the repo root on the box): bash tools/gpu_round.sh [tag] [pytest-args...]
TAG=${1:-r1}; shift
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }

timeout -k 10 500 python -m pytest tests -m gpu -q -rf "$@" > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a "$OUT/pytest_gpu_$TAG.log"; tail -5 "$OUT/pytest_gpu_$TAG.log"
ok $rc || exit $rc

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke_$TAG.log"
ok $rc || exit $rc

timeout -k 10 300 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench_$TAG.json"
[ $rc -eq 0 ] || { tail -20 "$OUT/bench_$TAG.err"; exit $rc; }

cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_$TAG" -o run \
    --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu > "$GRAFT_REPO_ROOT/$OUT/prof_$TAG.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
exit $rc
