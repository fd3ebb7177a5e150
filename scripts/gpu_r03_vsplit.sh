#!/bin/bash
# Vanilla per-graph (split) kernel: parity, bench (residue B=64, driver step counts), PMC traffic.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest tests/test_gpu_vanilla_fused.py tests/test_gpu_vanilla.py tests/test_gpu_distributed.py -q --timeout 120 --timeout-method thread > gpurun_out/r03/pt_vsplit.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -v amdgpu.ids gpurun_out/r03/pt_vsplit.log | tail -15
[ $rc -eq 0 ] || exit $rc
out=gpurun_out/r03/bench_vsplit.jsonl; : > $out
for i in 1 2; do
  timeout -k 10 200 python bench.py --model vanilla --graphs residue --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r03/b.log 2>&1; rc=$?
  echo "run $i rc=$rc: $(grep '^{' gpurun_out/r03/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["roofline"]["kernel_ms_avg"])')"
  grep '^{' gpurun_out/r03/b.log >> $out
  [ $rc -eq 0 ] || { tail -5 gpurun_out/r03/b.log; exit $rc; }
done
timeout -k 10 400 bash scripts/gpu_pmc_traffic.sh vanilla
