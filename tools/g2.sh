export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_product_wavefront.py tests/test_gpu_li.py tests/test_gpu_product.py tests/test_gpu_wavefront.py tests/test_gpu_batched.py -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/pytest_r3b.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_r3b.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --no-cpu --no-large-k > gpurun_out/bench_r3b.json 2> gpurun_out/bench_r3b.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_r3b.err
