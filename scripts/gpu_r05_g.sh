#!/bin/bash
# r05: pipelined GINet step: its tests, then the A/B against the two-launch step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05g; mkdir -p $O
: timeout -k 10 300 python -u -m pytest tests/test_gpu_train_step.py -x -v --timeout 120 --timeout-method thread > $O/pytest_step.log 2>&1; rc=$?
rc=0
bash scripts/gpu_ab.sh r05g/ab "-" "--model ginet;--model ginet --piped" 3 || exit $?
