#!/bin/bash
# PMC of the guide kernels on the Cornell K=128 line, per library build.
export PMC_SCRIPT=tools/cornell_bench.py
export PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"
SDMM_LIB_PATH=$GRAFT_REPO_ROOT/sdmm-mitsuba_amd/lib/libsdmm_amd.so bash tools/gpu_pmc.sh g16 --K 128 --modes 0 || exit 1
SDMM_LIB_PATH=$GRAFT_REPO_ROOT/sdmm-mitsuba_amd/build_ab/gg4.so bash tools/gpu_pmc.sh g4 --K 128 --modes 0 || exit 1
for t in g16 g4; do
  for k in guide_group_fallback guide_tree_cand_kernel; do
    python3 tools/pmc_summary.py gpurun_out/pmc_$t $k --K 128 --N 1 > gpurun_out/pmcsum_${t}_$k.json 2>&1
  done
  rm -rf gpurun_out/pmc_$t
done
