#!/bin/bash
# HBM traffic passes (FETCH_SIZE, WRITE_SIZE: one counter per run, no tracing) for
# the per-graph kernels: bash scripts/gpu_pmc_traffic.sh [model...] (default: foutnet sgat)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for M in ${@:-foutnet sgat}; do
  case $M in vanilla) K=vanilla_graph_kernel ;; ginet) K=ginet_graph_kernel ;; *) K=fout_graph_kernel ;; esac
  mkdir -p $R/gpurun_out/pmc_t_$M
  i=0
  for set in FETCH_SIZE WRITE_SIZE GRBM_GUI_ACTIVE; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set -f csv -d $R/gpurun_out/pmc_t_$M/p$i -o run -- python3 $R/tools/pmc_run.py 40 $M > $R/gpurun_out/pmc_t_$M/p$i.log 2>&1
    rc=$?; echo "$M pass $i ($set) rc=$rc"
    [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/pmc_t_$M/p$i.log; exit $rc; }
  done
  (cd $R && python3 tools/pmc_summary.py gpurun_out/pmc_t_$M $K > gpurun_out/pmc_${M}_graph_kernel.txt; cat gpurun_out/pmc_${M}_graph_kernel.txt; grep alg_bytes gpurun_out/pmc_t_$M/p1.log)
done
