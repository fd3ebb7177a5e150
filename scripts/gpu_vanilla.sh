#!/bin/bash
# VanillaNetwork per-graph kernel: parity tests, phase stamps, bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_vanilla_fused.py tests/test_gpu_vanilla.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_vanilla.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -v amdgpu.ids gpurun_out/pytest_vanilla.log | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python tools/stamp_profile.py 64 vanilla > gpurun_out/stamps_vanilla.log 2>&1; rc=$?
echo "stamps rc=$rc"; grep -v amdgpu.ids gpurun_out/stamps_vanilla.log | tail -22
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --model vanilla --graphs residue > gpurun_out/bench_vanilla.log 2>&1; rc=$?
echo "bench rc=$rc"; grep '^{' gpurun_out/bench_vanilla.log | cut -c1-250; grep '^{' gpurun_out/bench_vanilla.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline'])"
exit $rc
