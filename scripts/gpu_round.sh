#!/bin/bash
# GPU session script: tests -> smoke -> bench -> rocprof kernel trace. Stops at the first crash.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 420 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
ok $rc || exit $rc
timeout -k 10 240 python bench.py --steps 100 --warmup 10 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
ok $rc || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof" -o run -- python3 "${GRAFT_REPO_ROOT:-/root/repo}/bench.py" --steps 100 --warmup 10 --no-cpu-baseline > "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof.log" 2>&1; rc=$?; echo "rocprof rc=$rc"
find "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof" -name "*stats*"
exit $rc
