#!/bin/bash
# PMC passes (one counter group per run, no tracing domains) for the graph kernel.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_SMEM" \
           "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $set -f csv -d $R/gpurun_out/pmc/p$i -o run -- python3 $R/tools/pmc_run.py 40 > $R/gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc ($set)"
  [ $rc -eq 0 ] || exit $rc
done
