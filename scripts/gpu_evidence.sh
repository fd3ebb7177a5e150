#!/bin/bash
# Round evidence: GPU tests, smoke, headline bench (with CPU baseline), other
# configs, rocprofv3 kernel stats of the headline bench and of the vanilla run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -v amdgpu.ids gpurun_out/pytest_gpu.log | tail -4
[ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; grep '^{' gpurun_out/bench.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1; rc=$?
echo "bench (driver step counts) rc=$rc"; grep '^{' gpurun_out/bench_driver.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
[ -n "$SKIP_CONFIGS" ] || bash scripts/gpu_configs.sh || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline > $R/gpurun_out/prof.log 2>&1; rc=$?
echo "rocprof bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_vanilla -o run -- python3 $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline --model vanilla > $R/gpurun_out/prof_vanilla.log 2>&1; rc=$?
echo "rocprof vanilla rc=$rc"
find $R/gpurun_out/prof $R/gpurun_out/prof_vanilla -name "*kernel_stats*"
exit $rc
