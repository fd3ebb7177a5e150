#!/bin/bash
# One-launch step quick loop: bit-identity tests, epilogue stamps, default bench (200 steps).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_train_step.py tests/test_gpu_trainer.py -x -q --timeout 100 --timeout-method thread > gpurun_out/pt_sq.log 2>&1; rc=$?; tail -2 gpurun_out/pt_sq.log; grep -E "state after|Error" gpurun_out/pt_sq.log | cut -c1-300 | head -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python tools/step_stamps.py 64 > gpurun_out/ss.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ss.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-stream-copy > gpurun_out/b.log 2>&1; rc=$?
grep "^{" gpurun_out/b.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print("bench", r["value"], r["ms_per_step"], r["roofline"]["kernel_ms_avg"], r["roofline"]["frac"])'
exit $rc
