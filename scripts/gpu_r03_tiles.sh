#!/bin/bash
# Vanilla pipeline halo tiles: parity tests, then atom / mixed bench lines for
# tile sizes 64 / 32 / 128 / untiled, then rocprof kernel stats of the atom run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest tests/test_gpu_vanilla.py tests/test_gpu_vanilla_fused.py -q --timeout 120 --timeout-method thread > gpurun_out/r03/pt_vanilla.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -v amdgpu.ids gpurun_out/r03/pt_vanilla.log | tail -45
[ $rc -eq 0 ] || exit $rc
out=gpurun_out/r03/bench_tiles.jsonl; : > $out
for t in 32 16 64 0; do
  for g in atom mixed; do
    DR_VANILLA_TILE=$t timeout -k 10 200 python bench.py --steps 50 --warmup 5 --model vanilla --graphs $g --no-cpu-baseline > gpurun_out/r03/b.log 2>&1; rc=$?
    echo "tile=$t $g rc=$rc: $(grep '^{' gpurun_out/r03/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
    grep '^{' gpurun_out/r03/b.log | sed "s/^{/{\"tile\": $t, /" >> $out
    [ $rc -eq 0 ] || exit $rc
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/r03/prof_vatom -o run -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline --model vanilla --graphs atom > $R/gpurun_out/r03/prof_vatom.log 2>&1; rc=$?
echo "rocprof rc=$rc"; exit $rc
