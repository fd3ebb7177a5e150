#!/bin/bash
# FoutNet / SGAT per-graph kernel: parity, bench (configs[2], SGAT residue), stamps.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03
timeout -k 10 400 python -u -m pytest tests/test_gpu_foutnet.py tests/test_gpu_sgat.py tests/test_gpu_fout_large.py tests/test_gpu_mixed.py tests/test_gpu_layered.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r03/pt_fout.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -v amdgpu.ids gpurun_out/r03/pt_fout.log | tail -4; [ $rc -eq 0 ] || exit $rc
for m in foutnet sgat; do
  timeout -k 10 200 python bench.py --model $m --graphs residue --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r03/b.log 2>&1; rc=$?
  echo "$m rc=$rc: $(grep '^{' gpurun_out/r03/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["roofline"]["kernel_ms_avg"])')"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/r03/b.log; exit $rc; }
done
DR_LIB_NAME=libdeeprank2_amd_stamps.so timeout -k 10 200 python tools/stamp_profile.py 64 foutnet > gpurun_out/r03/stamps_fout.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r03/stamps_fout.txt; exit $rc
