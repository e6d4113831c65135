export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_r3c.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_r3c.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r3c.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_r3c.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r3c.json 2> gpurun_out/bench_r3c.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_r3c.err
