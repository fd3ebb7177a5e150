#!/bin/bash
# GPU session check: parity tests -> smoke -> headline bench -> extra bench configs given as args
# (each arg one quoted set of bench.py flags). Stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ]; }
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -v amdgpu.ids gpurun_out/pytest_gpu.log | tail -15
ok $rc || exit $rc
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
ok $rc || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; grep '^{' gpurun_out/bench.log | cut -c1-600
ok $rc || exit $rc
: > gpurun_out/bench_extra.jsonl
for cfg in "$@"; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline $cfg > gpurun_out/bench_cfg.log 2>&1; rc=$?
  echo "== [$cfg] rc=$rc"; grep '^{' gpurun_out/bench_cfg.log | tee -a gpurun_out/bench_extra.jsonl | cut -c1-300
  ok $rc || { tail -20 gpurun_out/bench_cfg.log; exit $rc; }
done
