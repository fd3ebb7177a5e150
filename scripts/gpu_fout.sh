#!/bin/bash
# FoutNet / SGAT iteration: parity tests, phase stamps, bench lines. Stops at the first crash.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_foutnet.py tests/test_gpu_sgat.py tests/test_gpu_layered.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_fout.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_fout.log
ok $rc || exit $rc
for m in foutnet sgat; do
  timeout -k 10 200 python tools/stamp_profile.py 64 $m > gpurun_out/stamps_$m.log 2>&1; rc=$?; echo "stamps $m rc=$rc"; grep -v amdgpu.ids gpurun_out/stamps_$m.log
  ok $rc || exit $rc
done
for m in foutnet sgat; do
  timeout -k 10 240 python bench.py --model $m --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench_$m.log 2>&1; rc=$?; echo "bench $m rc=$rc"; grep '^{' gpurun_out/bench_$m.log | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
  [ $rc -eq 0 ] || exit $rc
done
