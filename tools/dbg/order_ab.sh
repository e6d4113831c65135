for o in 1 0; do
  echo "== tree order $o"
  SDMM_TREE_ORDER=$o timeout -k 10 200 python tools/cornell_bench.py --K 16 128 --modes 0 > gpurun_out/to_$o.log 2>&1 || exit 1
  python3 tools/corn_summary.py < gpurun_out/to_$o.log
done
