# Phase laps (SDMM_GUIDING_TIMING) of the Cornell guided renders at K=16 and K=128
SDMM_GUIDING_TIMING=1 timeout -k 10 200 python tools/cornell_bench.py --K 16 128 --modes 0 > gpurun_out/laps.log 2>&1 || exit 1
python3 tools/corn_summary.py < gpurun_out/laps.log
