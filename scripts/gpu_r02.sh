#!/bin/bash
# Round-2 GPU session: parity tests -> smoke -> default bench -> extra bench lines.
# Stops at the first crash / timeout (exit codes other than 0/1 end the script).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 540 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu.log | tail -15
ok $rc || exit $rc
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
ok $rc || exit $rc
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_default.log 2>&1; rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_default.log | cut -c1-600
ok $rc || exit $rc
for extra in ${BENCH_EXTRA:-}; do
  args=$(echo "$extra" | tr ',' ' ')
  timeout -k 10 240 python bench.py --steps 50 --warmup 10 --no-cpu-baseline $args > "gpurun_out/bench_${extra//[, -]/_}.log" 2>&1; rc=$?; echo "bench $args rc=$rc"; grep -v amdgpu.ids "gpurun_out/bench_${extra//[, -]/_}.log" | cut -c1-400
  ok $rc || exit $rc
done
exit 0
