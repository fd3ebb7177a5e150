#!/bin/bash
# Vanilla chunk kernels: bench lines, then SQ counter passes (issue / wait / LDS) on atom-level B=32.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r04; mkdir -p $O/pmc_vc
timeout -k 10 300 python -u -m pytest tests/test_gpu_vanilla.py tests/test_gpu_vanilla_fused.py tests/test_gpu_mixed.py -x -q --timeout 120 --timeout-method thread > $O/pt_pmcvc.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pt_pmcvc.log; [ $rc -eq 0 ] || exit $rc
for g in atom mixed; do
  timeout -k 10 240 python bench.py --model vanilla --graphs $g --steps 60 --warmup 6 --no-cpu-baseline --no-stream-copy > $O/bench_vc4_$g.json 2> $O/bench_vc4_$g.err; rc=$?
  echo "vanilla $g rc=$rc: $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["ms_per_step"], d.get("step_split_us",{}).get("graph_pass"))' $O/bench_vc4_$g.json)"; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_vc4_atom -o run -- python3 $R/tools/pmc_run.py 20 vanilla_atom > $O/prof_vc4_atom.log 2>&1; rc=$?
echo "kernel-trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find $O/prof_vc4_atom -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | cut -c1-110 | sed -n 1,10p
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -f csv -d $O/pmc_vc/p$i -o run -- python3 $R/tools/pmc_run.py 6 vanilla_atom > $O/pmc_vc/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $O/pmc_vc/p$i.log; exit $rc; }
done
cd $R
for k in "vc_fwd<3, 1>" "vc_fwd<3, 2>" "vc_eb2n1" "vc_eb1" "vc_nb2" "vb_head" "vc_combine"; do echo "== $k"; python3 tools/pmc_summary.py $O/pmc_vc "$k"; done > $O/pmc_vc_summary.txt
cat $O/pmc_vc_summary.txt | head -120
