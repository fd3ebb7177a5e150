#!/bin/bash
# r05: accumulating pass, prefetched staging without the store-ack wait — suite, acc stamps, A/B vs HEAD.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05u; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_gpu.log | head -20; exit $rc; }
DR_ACC_PREFETCH=1 timeout -k 10 300 python tools/acc_stamps.py 4096 > $O/stamps_pf.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/stamps_pf.txt
bash scripts/gpu_ab.sh r05u/ab "base -" "--batch 4096 --batches 2 --acc on;--model ginet" 3
