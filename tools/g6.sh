export TMPDIR=/tmp; mkdir -p gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_prod" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/cornell_bench.py" --K 16 --modes 0 --product > "$GRAFT_REPO_ROOT/gpurun_out/prof_prod.log" 2>&1
rc=$?; echo "prof product rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_k128" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/cornell_bench.py" --K 128 --modes 0 > "$GRAFT_REPO_ROOT/gpurun_out/prof_k128.log" 2>&1
rc=$?; echo "prof k128 rc=$rc"
