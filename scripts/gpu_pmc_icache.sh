#!/bin/bash
# Instruction-cache PMC of ginet_graph_kernel for several library variants:
#   bash scripts/gpu_pmc_icache.sh <out-subdir> "<lib suffixes>" ["<counter set>" ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${1:-icache}; mkdir -p $O
read -ra VARS <<< "$2"; shift 2
SETS=("$@"); [ ${#SETS[@]} -eq 0 ] && SETS=("SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM")
export TMPDIR=/tmp
for v in "${VARS[@]}"; do
  lib=libdeeprank2_amd.so; [ "$v" != "-" ] && lib=libdeeprank2_amd_$v.so
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1)); d=$O/$v/p$i; mkdir -p $O/$v
    (cd /tmp && DR_LIB_NAME=$lib timeout -s KILL 90 rocprofv3 --pmc $set -f csv -d $d -o run -- python3 $R/tools/pmc_run.py 40 ginet > $d.log 2>&1); rc=$?
    echo "$v pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $d.log; exit $rc; }
  done
  echo "== $v"; python3 tools/pmc_summary.py $O/$v ginet_graph_kernel | tee $O/summary_$v.txt
done
