#!/bin/bash
# GINet kernel iteration: GINet parity tests, stamp profile, default bench (driver's step counts).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_ginet.py tests/test_gpu_large.py tests/test_gpu_trainer.py tests/test_gpu_mixed.py -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_iter.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/stamp_profile.py 64 > gpurun_out/stamps.log 2>&1; rc=$?; echo "stamps rc=$rc"; grep -v amdgpu.ids gpurun_out/stamps.log
ok $rc || exit $rc
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-stream-copy > gpurun_out/bench_iter.log 2>&1; rc=$?; echo "bench rc=$rc"; grep "^{" gpurun_out/bench_iter.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["roofline"]["kernel_ms_avg"])'
timeout -k 10 240 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-stream-copy > gpurun_out/bench_iter200.log 2>&1; rc=$?; echo "bench200 rc=$rc"; grep "^{" gpurun_out/bench_iter200.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["roofline"]["kernel_ms_avg"])'
exit $rc
