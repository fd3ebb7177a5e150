#!/bin/bash
# r04 second batch:
#  * reduce-at-start (RAS) GINet step: bit-identity tests + configs[1] bench default vs --ras
#  * per-kernel HBM traffic (FETCH_SIZE / WRITE_SIZE) of the Vanilla paths at HEAD: per-graph (residue B=64),
#    chunk-fused pipeline (atom B=32, mixed B=64)
#  * the batch-size sweep of the headline step
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
O=$R/gpurun_out/r04
mkdir -p $O
for W in atom mixed; do
  DR_LIB_NAME=libdeeprank2_amd_stamps.so timeout -k 10 120 python tools/vchunk_stamps.py $W > $O/vchunk_stamps_$W.txt 2>&1; rc=$?
  echo "stamps $W rc=$rc"; cat $O/vchunk_stamps_$W.txt | grep -v amdgpu.ids | cut -c1-400; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_step.py -x -v --timeout 120 --timeout-method thread > $O/pt_ras.log 2>&1; rc=$?
echo "pytest train_step rc=$rc"; grep -E "passed|failed|Error" $O/pt_ras.log | tail -5; [ $rc -eq 0 ] || exit $rc
for M in "" "--ras"; do
  n=default; [ -n "$M" ] && n=ras
  timeout -k 10 240 python bench.py --steps 400 --warmup 20 --no-cpu-baseline $M > $O/bench_ginet_$n.json 2> $O/bench_ginet_$n.err; rc=$?
  echo "ginet $n rc=$rc: $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["ms_per_step"], d.get("step_split_us"))' $O/bench_ginet_$n.json)"; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp
for W in vanilla vanilla_atom vanilla_mixed; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/kt2_$W -o run -- python3 $R/tools/pmc_run.py 20 $W > $O/kt2_$W.log 2>&1
  rc=$?; echo "$W kernel-trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/kt2_$W.log; exit $rc; }
  for set in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $set -f csv -d $O/pmc2_$W/$set -o run -- python3 $R/tools/pmc_run.py 20 $W > $O/pmc2_${W}_$set.log 2>&1
    rc=$?; echo "$W $set rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/pmc2_${W}_$set.log; exit $rc; }
  done
  f=$(find $O/kt2_$W -name "*kernel_stats.csv" | head -1)
  (cd $R && python3 tools/pmc_per_kernel.py $O/pmc2_$W "$f" 20 > $O/pmc_per_kernel_${W}_r04.txt; cut -c1-130 $O/pmc_per_kernel_${W}_r04.txt)
done
cd $R
out=$O/batch_sweep_ginet.jsonl
: > $out
for B in 64 256 1024 4096 16384; do
  nb=4; [ $B -ge 4096 ] && nb=2; [ $B -ge 16384 ] && nb=1
  timeout -k 10 400 python bench.py --batch $B --batches $nb --steps 20 --warmup 3 --no-cpu-baseline > $O/sweep.log 2>&1; rc=$?
  echo "== B=$B rc=$rc"
  grep '^{' $O/sweep.log | tee -a $out | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_ms_avg'], r['achieved'], r['frac'])"
  [ $rc -eq 0 ] || { tail -5 $O/sweep.log; exit $rc; }
done
