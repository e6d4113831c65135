#!/bin/bash
# One GPU-box session: selected GPU tests (ordinary failures, rc 1, let the
# session go on; a fault / abort / timeout ends it), then the responsibility
# E-step A/B over library variants.
# Usage: bash tools/gpu_session.sh TAG "pytest targets" "lib1.so lib2.so ..."
TAG=$1; TESTS=$2; LIBS=$3
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -q -rf --timeout 300 --timeout-method thread \
      > $OUT/pytest_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 $OUT/pytest_$TAG.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
if [ -n "$LIBS" ]; then
  bash tools/gpu_resp_ab.sh "$LIBS" 0
fi
