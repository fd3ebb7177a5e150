#!/bin/bash
# Default bench at the driver's step counts, rest-graph on/off, plus 200 steps.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for cfg in "1 20 5" "0 20 5" "1 20 5" "1 200 20"; do
  set -- $cfg
  DR_BENCH_REST=$1 timeout -k 10 200 python bench.py --steps $2 --warmup $3 --no-cpu-baseline --no-stream-copy > gpurun_out/bm.log 2>&1; rc=$?
  echo "rest=$1 steps=$2: $(grep '^{' gpurun_out/bm.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["roofline"]["kernel_ms_avg"], r["launch"])')"
  [ $rc -eq 0 ] || exit $rc
done
