#!/bin/bash
# r04 baseline measurements at HEAD:
#  * Vanilla pipeline per-kernel HBM traffic (FETCH_SIZE / WRITE_SIZE passes) + kernel stats, atom B=32 and mixed B=64
#  * GINet atom-level fp32 / bf16 step split (rocprof kernel stats of the bench run)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
O=$R/gpurun_out/r04
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for W in vanilla_atom vanilla_mixed; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/kt_$W -o run -- python3 $R/tools/pmc_run.py 20 $W > $O/kt_$W.log 2>&1
  rc=$?; echo "$W kernel-trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/kt_$W.log; exit $rc; }
  for set in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $set -f csv -d $O/pmc_$W/$set -o run -- python3 $R/tools/pmc_run.py 20 $W > $O/pmc_${W}_$set.log 2>&1
    rc=$?; echo "$W $set rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/pmc_${W}_$set.log; exit $rc; }
  done
  f=$(find $O/kt_$W -name "*kernel_stats.csv" | head -1)
  (cd $R && python3 tools/pmc_per_kernel.py $O/pmc_$W "$f" 20 > $O/pmc_per_kernel_$W.txt; cat $O/pmc_per_kernel_$W.txt | cut -c1-130)
done
for D in f32 bf16; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $O/kt_ginet_atom_$D -o run -- python3 $R/bench.py --model ginet --graphs atom --dtype $D --steps 100 --warmup 10 --no-cpu-baseline --no-stream-copy > $O/kt_ginet_atom_$D.log 2>&1
  rc=$?; echo "ginet atom $D rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/kt_ginet_atom_$D.log; exit $rc; }
  f=$(find $O/kt_ginet_atom_$D -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | cut -c1-120 | sed -n 1,10p
  grep '^{' $O/kt_ginet_atom_$D.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms_avg"])'
done
