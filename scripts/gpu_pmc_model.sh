#!/bin/bash
# PMC passes for one model's graph kernel: bash scripts/gpu_pmc_model.sh <ginet|vanilla> [pass-set...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); M=${1:-vanilla}
mkdir -p gpurun_out/pmc_$M
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR" \
           "SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_SENDMSG"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -f csv -d $R/gpurun_out/pmc_$M/p$i -o run -- python3 $R/tools/pmc_run.py 20 $M > $R/gpurun_out/pmc_$M/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/pmc_$M/p$i.log; exit $rc; }
done
cd $R && python3 tools/pmc_summary.py gpurun_out/pmc_$M ${2:-vanilla_graph_kernel}
