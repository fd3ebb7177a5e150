#!/bin/bash
# One-launch step: bit-identity test, then kernel time with the reduction (handoff 1) and without (9, diagnostic).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_train_step.py -x -q --timeout 100 --timeout-method thread > gpurun_out/pt_handoff.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error|state after" gpurun_out/pt_handoff.log | cut -c1-600 | tail -4
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for m in 1 9; do
  DR_STEP_HANDOFF=$m timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-stream-copy > gpurun_out/bench_handoff$m.log 2>&1; rc=$?
  echo "handoff $m bench rc=$rc"; grep "^{" gpurun_out/bench_handoff$m.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["roofline"]["kernel_ms_avg"], r["roofline"]["frac"])'
  [ $rc -eq 0 ] || exit $rc
done
