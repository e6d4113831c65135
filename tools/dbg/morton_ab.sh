for b in 10 7 5; do
  echo "== bits $b"
  SDMM_MORTON_BITS=$b timeout -k 10 200 python tools/cornell_bench.py --K 16 128 --modes 0 > gpurun_out/mb_$b.log 2>&1 || exit 1
  python3 tools/corn_summary.py < gpurun_out/mb_$b.log
done
