#!/bin/bash
# r05: isolated A/B of each GINet change first, then the GPU suite, then stamps.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05d; mkdir -p $O
bash scripts/gpu_ab.sh r05d/ab "base - onlyfc1 onlyhead headdpp onlypf onlycl1" "--model ginet" 2 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_gpu.log | head -20; exit $rc; }
bash scripts/gpu_r05_evidence.sh r05d/ev stamps
