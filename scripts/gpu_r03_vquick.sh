#!/bin/bash
# Vanilla per-graph kernel: stamps + residue bench (quick iteration).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03
DR_LIB_NAME=libdeeprank2_amd_stamps.so timeout -k 10 200 python tools/stamp_profile.py 64 vanilla > gpurun_out/r03/stamps_vanilla.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r03/stamps_vanilla.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -m pytest tests/test_gpu_vanilla_fused.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r03/pt_vq.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r03/pt_vq.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python bench.py --model vanilla --graphs residue --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r03/b.log 2>&1; rc=$?
  echo "run $i rc=$rc: $(grep '^{' gpurun_out/r03/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["roofline"]["kernel_ms_avg"])')"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/r03/b.log; exit $rc; }
done
