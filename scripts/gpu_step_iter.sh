#!/bin/bash
# One-launch GINet step: its bit-identity tests, the GINet/trainer parity tests, default bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_step.py tests/test_gpu_ginet.py tests/test_gpu_trainer.py tests/test_gpu_mixed.py tests/test_gpu_distributed.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_step.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_step.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-stream-copy > gpurun_out/bench_step20.log 2>&1; rc=$?; echo "bench20 rc=$rc"; grep "^{" gpurun_out/bench_step20.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["roofline"]["kernel_ms_avg"], r["roofline"]["frac"])'
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-stream-copy > gpurun_out/bench_step200.log 2>&1; rc=$?; echo "bench200 rc=$rc"; grep "^{" gpurun_out/bench_step200.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["roofline"]["kernel_ms_avg"], r["roofline"]["frac"])'
exit $rc
