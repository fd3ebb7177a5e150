#!/bin/bash
# r05: LDS bank-conflict counters of the headline kernel (ginet_graph_kernel, B=64).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r05lds; mkdir -p $O
export TMPDIR=/tmp
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -f csv -d $O/p1 -o run -- python3 $R/tools/pmc_run.py 40 ginet > $O/p1.log 2>&1); rc=$?
echo "pmc rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/p1.log; exit $rc; }
python3 tools/pmc_summary.py $O ginet_graph_kernel > $O/pmc_lds_ginet.txt; cat $O/pmc_lds_ginet.txt
