#!/bin/bash
# Quick GPU iteration: parity tests, stamp profile, short bench. Stops at the first crash.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 300 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 200 python tools/stamp_profile.py 64 > gpurun_out/stamps.log 2>&1; rc=$?; echo "stamps rc=$rc"; grep -v amdgpu.ids gpurun_out/stamps.log
ok $rc || exit $rc
timeout -k 10 240 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench.log | cut -c1-400
exit $rc
