export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_corn128 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/cornell_bench.py --K 128 --modes 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_corn128.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_corn512p -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/cornell_bench.py --K 512 --modes 0 --product > $GRAFT_REPO_ROOT/gpurun_out/prof_corn512p.log 2>&1
