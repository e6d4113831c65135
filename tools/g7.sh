export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_product.py tests/test_gpu_product_wavefront.py tests/test_gpu_li_oracle.py tests/test_gpu_li.py -m gpu -q -rf -x --timeout 120 --timeout-method thread > gpurun_out/pytest_r3f.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_r3f.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/cornell_bench.py --K 16 --modes 0 --product > gpurun_out/cornell_r3f.log 2>&1
rc=$?; echo "cornell rc=$rc"; grep workload gpurun_out/cornell_r3f.log | cut -c1-200
