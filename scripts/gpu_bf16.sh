#!/bin/bash
# bf16 (configs[3]) session: bf16 + mixed parity tests, atom-level bench lines fp32/bf16, rocprof of the bf16 step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_mixed.py tests/test_gpu_large.py -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_bf16.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_bf16.log | tail -15
ok $rc || exit $rc
for dt in f32 bf16; do
  timeout -k 10 240 python bench.py --graphs atom --dtype $dt --steps 40 --warmup 8 --no-cpu-baseline > gpurun_out/bench_atom_$dt.log 2>&1; rc=$?; echo "bench atom $dt rc=$rc"; grep "^{" gpurun_out/bench_atom_$dt.log | cut -c1-300
  ok $rc || exit $rc
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof_atom_bf16" -o run -- python3 "${GRAFT_REPO_ROOT:-/root/repo}/bench.py" --graphs atom --dtype bf16 --steps 40 --warmup 8 --no-cpu-baseline --no-stream-copy > "${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof_atom_bf16.log" 2>&1; rc=$?; echo "rocprof rc=$rc"
exit $rc
