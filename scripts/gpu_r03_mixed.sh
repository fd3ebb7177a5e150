#!/bin/bash
# Mixed-batch dispatch (per-graph kernel + large path on two streams): parity, bench lines, rocprof.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out/r03
timeout -k 10 400 python -u -m pytest tests/test_gpu_mixed.py tests/test_gpu_large.py tests/test_gpu_fout_large.py tests/test_gpu_ginet.py -q --timeout 120 --timeout-method thread > gpurun_out/r03/pt_mixed.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -v amdgpu.ids gpurun_out/r03/pt_mixed.log | tail -30
[ $rc -eq 0 ] || exit $rc
out=gpurun_out/r03/bench_mixed.jsonl; : > $out
for cfg in "--model ginet --graphs mixed" "--model foutnet --graphs mixed" "--model sgat --graphs mixed"; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 $cfg --no-cpu-baseline > gpurun_out/r03/b.log 2>&1; rc=$?
  echo "$cfg rc=$rc: $(grep '^{' gpurun_out/r03/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  grep '^{' gpurun_out/r03/b.log >> $out
  [ $rc -eq 0 ] || { tail -5 gpurun_out/r03/b.log; exit $rc; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/r03/prof_gmixed -o run -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline --model ginet --graphs mixed > $R/gpurun_out/r03/prof_gmixed.log 2>&1; rc=$?
echo "rocprof rc=$rc"; exit $rc
