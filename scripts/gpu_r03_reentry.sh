#!/bin/bash
# Re-entry check of the rebuilt library: every GPU test, smoke, default bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03/pytest_gpu_reentry.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r03/pytest_gpu_reentry.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python __graft_entry__.py smoke > gpurun_out/r03/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/r03/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03/bench_reentry.json 2> gpurun_out/r03/bench_reentry.err; rc=$?
echo "bench rc=$rc"; cut -c1-600 gpurun_out/r03/bench_reentry.json
exit $rc
[ $rc -eq 0 ] || exit $rc
for g in atom mixed; do
  timeout -k 10 240 python bench.py --model vanilla --graphs $g --steps 60 --warmup 6 --no-cpu-baseline > gpurun_out/r03/bench_vanilla_$g.json 2> gpurun_out/r03/bench_vanilla_$g.err; rc=$?
  echo "vanilla $g rc=$rc: $(cut -c1-300 gpurun_out/r03/bench_vanilla_$g.json)"; [ $rc -eq 0 ] || exit $rc
done
R=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/r03/prof_vatom -o run -- python3 $R/bench.py --model vanilla --graphs atom --steps 60 --warmup 6 --no-cpu-baseline --no-stream-copy > $R/gpurun_out/r03/prof_vatom.log 2>&1; rc=$?
echo "rocprof rc=$rc"
exit $rc
