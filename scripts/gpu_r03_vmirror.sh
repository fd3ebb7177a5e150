#!/bin/bash
# Vanilla packed-weight mirror (Adam rewrites the fragment-order copy): parity + residue bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03
timeout -k 10 400 python -u -m pytest tests/test_gpu_vanilla_fused.py tests/test_gpu_vanilla.py tests/test_gpu_distributed.py tests/test_gpu_trainer.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r03/pt_vm.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r03/pt_vm.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python bench.py --model vanilla --graphs residue --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r03/b.log 2>&1; rc=$?
  echo "run $i rc=$rc: $(grep '^{' gpurun_out/r03/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["roofline"]["kernel_ms_avg"])')"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/r03/b.log; exit $rc; }
done
cp gpurun_out/r03/b.log gpurun_out/r03/bench_vanilla_mirror.log
