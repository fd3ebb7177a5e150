#!/bin/bash
# r05 first GPU call: the GPU suite on the new library, the headline A/B of the
# GINet staging / head changes, then the counter evidence at this tree.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh r05b/ab "base - noprefetch fc1early serialhead" "--model ginet" 2 || exit $?
bash scripts/gpu_r05_evidence.sh r05b/ev
