#!/bin/bash
# rocprofv3 PMC passes over tools/prof_kernels.py, one counter group per pass
# (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass; no
# tracing domains beside --pmc).  Each pass has its own time limit; the first
# failure ends the script.
# Usage (on the box, repo root): bash tools/gpu_pmc.sh TAG [prof_kernels args...]
TAG=${1:-r1}; shift
OUT="$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || { echo "counter listing failed"; exit 1; }
i=0
# PMC_GROUPS (optional): counter groups separated by ';' replace the default passes
GROUPS_DEFAULT="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU;SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_LDS;SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_MISC;GRBM_GUI_ACTIVE GRBM_COUNT"
IFS=';' read -r -a GROUP_LIST <<< "${PMC_GROUPS:-$GROUPS_DEFAULT}"
for group in "${GROUP_LIST[@]}"; do
  i=$((i + 1))
  timeout -k 10 240 rocprofv3 --pmc $group --output-format csv -d "$OUT/p$i" -o run \
      -- python3 "$GRAFT_REPO_ROOT/${PMC_SCRIPT:-tools/prof_kernels.py}" "$@" > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($group) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$OUT/p$i.log"; exit $rc; }
done
