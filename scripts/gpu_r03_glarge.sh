#!/bin/bash
# GINet tail on atom-level graphs: parity, atom / mixed / residue bench, large-tail stamps.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03
timeout -k 10 400 python -u -m pytest tests/test_gpu_ginet.py tests/test_gpu_large.py tests/test_gpu_train_step.py tests/test_gpu_mixed.py tests/test_gpu_bf16.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r03/pt_glarge.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -v amdgpu.ids gpurun_out/r03/pt_glarge.log | tail -3; [ $rc -eq 0 ] || exit $rc
for g in atom mixed residue; do
  timeout -k 10 200 python bench.py --model ginet --graphs $g --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r03/b.log 2>&1; rc=$?
  echo "$g rc=$rc: $(grep '^{' gpurun_out/r03/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["roofline"]["kernel_ms_avg"])')"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/r03/b.log; exit $rc; }
done
DR_LIB_NAME=libdeeprank2_amd_stamps.so timeout -k 10 200 python tools/stamp_profile.py 32 ginet_large > gpurun_out/r03/stamps_glarge.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r03/stamps_glarge.txt; exit $rc
