#!/bin/bash
# Batch-size sweep of the headline GINet step: graphs/s and the
# graph pass's HBM roofline fraction from B=64 (configs[1]) up to 16384 graphs.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/batch_sweep.jsonl
: > $out
for B in 64 256 1024 4096 16384; do
  nb=4; [ $B -ge 4096 ] && nb=2; [ $B -ge 16384 ] && nb=1
  timeout -k 10 400 python bench.py --batch $B --batches $nb --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/sweep.log 2>&1; rc=$?
  echo "== B=$B rc=$rc"
  grep '^{' gpurun_out/sweep.log | tee -a $out | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_ms_avg'], r['achieved'], r['frac'])"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/sweep.log; exit $rc; }
done
