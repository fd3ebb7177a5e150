#!/bin/bash
# r05 final: GPU suite + smoke, headline A/B against the pre-accumulating-pass
# library, the accumulating pass's batch sweep (prefetch on / off, per-graph
# partials), per-kernel HBM at B=4096, the headline PMC + rocprof stats at HEAD.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r05m; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh r05m/ab "prev -" "--model ginet" 3 || exit 1
: > $O/sweep.jsonl
for B in 64 256 1024 4096 16384; do
  nb=4; [ $B -ge 4096 ] && nb=2; [ $B -ge 16384 ] && nb=1
  for mode in "--acc off" "--acc on --no-acc-prefetch" "--acc on"; do
    [ $B -le 256 ] && [ "$mode" != "--acc off" ] && continue
    timeout -k 10 400 python bench.py --batch $B --batches $nb --steps 20 --warmup 3 --no-cpu-baseline --no-stream-copy $mode > $O/sweep.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { tail -5 $O/sweep.log; exit $rc; }
    echo "B=$B $mode | $(grep '^{' $O/sweep.log | tee -a $O/sweep.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d.get('step_split_us') or {}; print(round(d['value']), 'step_us', round(d['ms_per_step']*1000,2), 'pass_us', s.get('graph_pass'), 'reduce_us', s.get('reduce_adam'), 'frac', round(d['roofline']['frac'],4))")" | tee -a $O/sweep.txt
  done
done
# per-kernel HBM bytes of the accumulating step at B = 4096
W=ginet_b4096; n=6; mkdir -p $O/pmc_$W
(cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/kt_$W -o run -- python3 $R/tools/pmc_run.py $n $W > $O/kt_$W.log 2>&1) || { echo "kt rc=$?"; tail -5 $O/kt_$W.log; exit 1; }
for set in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $set -f csv -d $O/pmc_$W/$set -o run -- python3 $R/tools/pmc_run.py $n $W > $O/pmc_$W/$set.log 2>&1) || { echo "pmc $set failed"; exit 1; }
done
f=$(find $O/kt_$W -name "*kernel_stats.csv" | head -1)
python3 tools/pmc_per_kernel.py $O/pmc_$W "$f" $n > $O/pmc_per_kernel_$W.txt; cut -c1-120 $O/pmc_per_kernel_$W.txt | head -6
bash scripts/gpu_r05_evidence.sh r05m/ev pmc_headline bench
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt_headline -o run -- python3 $R/bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/kt_headline.log 2>&1); echo "headline rocprof rc=$?"
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $O/bench_default.json 2> $O/bench_default.err; rc=$?; echo "bench rc=$rc"; cut -c1-300 $O/bench_default.json
echo done
