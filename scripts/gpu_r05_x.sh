#!/bin/bash
# r05: FoutNet gather one row, two chunks per lane — suite, stamps, A/B vs HEAD.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05x; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_gpu.log | head -20; exit $rc; }
DR_LIB_NAME=libdeeprank2_amd_stamps.so timeout -k 10 200 python tools/stamp_profile.py 64 > $O/stamps.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/stamps.txt

bash scripts/gpu_ab.sh r05x/ab "base -" "--model foutnet;--model foutnet --graphs mixed" 3
