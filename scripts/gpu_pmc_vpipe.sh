#!/bin/bash
# PMC passes for the Vanilla pipeline's tiled edge kernels on atom-level graphs (B=32).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out/pmc_vpipe
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -f csv -d $R/gpurun_out/pmc_vpipe/p$i -o run -- python3 $R/tools/pmc_run.py 6 vanilla_atom > $R/gpurun_out/pmc_vpipe/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/pmc_vpipe/p$i.log; exit $rc; }
done
cd $R
for k in vb_edge_fwd_tile vb_edge_bwd_tile vb_wgrad_mfma; do echo "== $k"; python3 tools/pmc_summary.py gpurun_out/pmc_vpipe $k; done
