#!/bin/bash
# Round-3 first GPU session: tests, the driver's bench command, and the MFMA
# utilisation PMC passes for the GINet and Vanilla graph kernels.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r03/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03/bench_driver.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -c 600 gpurun_out/r03/bench_driver.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > $R/gpurun_out/r03/pmc_avail.txt 2>&1; echo "list-avail rc=$?"
bash $R/scripts/gpu_pmc_mfma.sh ginet vanilla
