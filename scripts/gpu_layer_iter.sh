#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_layered.py tests/test_gpu_nonfinite.py tests/test_gpu_foutnet.py tests/test_gpu_sgat.py tests/test_gpu_ginet_nocluster.py tests/test_gpu_mixed.py tests/test_gpu_ginet.py tests/test_gpu_pooling.py -x -q --timeout 150 --timeout-method thread > gpurun_out/pt_lay.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pt_lay.log | tail -6
[ $rc -eq 0 ] || exit $rc
for m in foutnet sgat ginet_nocluster; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-stream-copy --model $m --graphs mixed > gpurun_out/bl_$m.log 2>&1; rc=$?
  echo "$m mixed: $(grep '^{' gpurun_out/bl_$m.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
  [ $rc -eq 0 ] || exit $rc
done
