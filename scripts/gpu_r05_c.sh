#!/bin/bash
# r05: GPU suite on the new library, then the isolated A/B of each GINet change, then stamps.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/pytest_gpu.log | head -20; exit $rc; }
bash scripts/gpu_ab.sh r05c/ab "base - onlyfc1 onlyhead headdpp onlypf onlycl1" "--model ginet" 2 || exit $?
bash scripts/gpu_r05_evidence.sh r05c/ev stamps
