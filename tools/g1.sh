export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_r3a.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_r3a.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
SDMM_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --no-large-k > gpurun_out/rehearse_r3a.json 2> gpurun_out/rehearse_r3a.err
rc=$?; echo "rehearse rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/rehearse_r3a.err; exit $rc; }
timeout -k 10 300 python bench.py --no-extra --no-cpu > gpurun_out/bench_r3a.json 2> gpurun_out/bench_r3a.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_r3a.json
