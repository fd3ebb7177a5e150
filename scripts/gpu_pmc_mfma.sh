#!/bin/bash
# MFMA-utilisation PMC pass (one run per model, no tracing domains) for the
# per-graph kernels: bash scripts/gpu_pmc_mfma.sh [model...] (default: ginet vanilla)
# Counters: SQ_VALU_MFMA_BUSY_CYCLES (matrix-pipe busy cycles summed over SIMDs),
# SQ_INSTS_MFMA, SQ_BUSY_CU_CYCLES, SQ_BUSY_CYCLES, SQ_WAVE_CYCLES, GRBM_GUI_ACTIVE.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
SET="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CU_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
for M in ${@:-ginet vanilla}; do
  case $M in vanilla) K=vanilla_graph_kernel ;; ginet) K=ginet_graph_kernel ;; *) K=fout_graph_kernel ;; esac
  mkdir -p $R/gpurun_out/pmc_m_$M
  timeout -s KILL 90 rocprofv3 --pmc $SET -f csv -d $R/gpurun_out/pmc_m_$M/p1 -o run -- python3 $R/tools/pmc_run.py 40 $M > $R/gpurun_out/pmc_m_$M/p1.log 2>&1
  rc=$?; echo "$M mfma pass rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/pmc_m_$M/p1.log; exit $rc; }
  (cd $R && python3 tools/pmc_summary.py gpurun_out/pmc_m_$M $K > gpurun_out/pmc_mfma_${M}.txt; cat gpurun_out/pmc_mfma_${M}.txt)
done
