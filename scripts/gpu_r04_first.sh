#!/bin/bash
# r04 first GPU call: changed-path tests (edge-balanced DDP shards, trainer checkpoint epoch), then baseline measurements.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_trainer.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r04/pt_first.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/r04/pt_first.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r04_measure.sh
