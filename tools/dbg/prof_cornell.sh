# rocprofv3 kernel stats of one Cornell guided render (K per argument)
export TMPDIR=/tmp
K=${1:-16}
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_corn$K" -o run \
    --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/cornell_bench.py" --K $K --modes 0 > "$GRAFT_REPO_ROOT/gpurun_out/prof_corn$K.log" 2>&1
