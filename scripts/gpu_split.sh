#!/bin/bash
# Vanilla split kernel: Vanilla parity tests first, then the whole GPU suite, then residue / mixed bench lines.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_vanilla_fused.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pt_split.log 2>&1; rc=$?
echo "split tests rc=$rc"; grep -E "passed|failed|FAILED|Error|assert" gpurun_out/pt_split.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 540 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "gpu suite rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu.log | tail -8
[ $rc -eq 0 ] || exit $rc
for g in residue mixed; do
  timeout -k 10 240 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-stream-copy --model vanilla --graphs $g > gpurun_out/bv_$g.log 2>&1; rc=$?
  echo "vanilla $g: $(grep '^{' gpurun_out/bv_$g.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["roofline"]["kernel_ms_avg"], r["roofline"]["frac"])')"
  [ $rc -eq 0 ] || exit $rc
done
