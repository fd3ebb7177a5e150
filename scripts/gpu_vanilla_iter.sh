#!/bin/bash
# Vanilla iteration: parity tests, then atom / mixed / residue bench lines.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_vanilla.py tests/test_gpu_vanilla_fused.py tests/test_gpu_mixed.py -x -q --timeout 150 --timeout-method thread > gpurun_out/pt_van.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pt_van.log | tail -6
[ $rc -eq 0 ] || exit $rc
for g in atom mixed residue; do
  timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-stream-copy --model vanilla --graphs $g > gpurun_out/bv_$g.log 2>&1; rc=$?
  echo "vanilla $g: $(grep '^{' gpurun_out/bv_$g.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["roofline"]["kernel_ms_avg"], r["roofline"]["frac"])')"
  [ $rc -eq 0 ] || exit $rc
done
