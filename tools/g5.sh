export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_stree.py tests/test_gpu_li.py tests/test_gpu_harness.py tests/test_gpu_li_oracle.py -m gpu -q -rf -x --timeout 120 --timeout-method thread > gpurun_out/pytest_r3e.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -20 gpurun_out/pytest_r3e.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
SDMM_GUIDING_TIMING=1 timeout -k 10 300 python tools/cornell_bench.py --K 16 128 --modes 0 1 > gpurun_out/cornell_r3e.log 2>&1
rc=$?; echo "cornell rc=$rc"
