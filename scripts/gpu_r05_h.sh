#!/bin/bash
# r05: pipelined step timing (DR_STEP_DIAG 1: no waits, wrong results) and the reducer count
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05h; mkdir -p $O; : > $O/diag.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_step.py -x -q --timeout 120 --timeout-method thread -k piped > $O/pytest_step.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest_step.log; [ $rc -eq 0 ] || exit $rc
for cfg in "0 32" "1 32" "0 16" "0 64" "0 85"; do
  set -- $cfg
  DR_STEP_DIAG=$1 DR_PIPED_NR=$2 timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-stream-copy --piped > $O/b.log 2> $O/b.err; rc=$?
  [ $rc -eq 0 ] || { tail -5 $O/b.err; exit $rc; }
  echo "diag $1 NR $2 | $(grep '^{' $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("step_us", round(d["ms_per_step"]*1000,2), "kernel_us", round(d["roofline"]["kernel_ms_avg"]*1000,2))')" | tee -a $O/diag.txt
done
