#!/bin/bash
# FoutNet / SGAT large-graph kernels: parity, then mixed / atom bench lines, rocprof of FoutNet mixed.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest tests/test_gpu_fout_large.py tests/test_gpu_layered.py tests/test_gpu_foutnet.py tests/test_gpu_sgat.py -q --timeout 120 --timeout-method thread > gpurun_out/r03/pt_fout.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -v amdgpu.ids gpurun_out/r03/pt_fout.log | tail -40
[ $rc -eq 0 ] || exit $rc
out=gpurun_out/r03/bench_fout.jsonl; : > $out
for cfg in "--model foutnet --graphs mixed" "--model sgat --graphs mixed" "--model foutnet --graphs atom" "--model foutnet --graphs residue"; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 5 $cfg --no-cpu-baseline > gpurun_out/r03/b.log 2>&1; rc=$?
  echo "$cfg rc=$rc: $(grep '^{' gpurun_out/r03/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  grep '^{' gpurun_out/r03/b.log >> $out
  [ $rc -eq 0 ] || { tail -5 gpurun_out/r03/b.log; exit $rc; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/r03/prof_fmixed -o run -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline --model foutnet --graphs mixed > $R/gpurun_out/r03/prof_fmixed.log 2>&1; rc=$?
echo "rocprof rc=$rc"; exit $rc
