#!/bin/bash
# one-launch GINet path: parity (bit-identity to the two-launch path, oracle, capture), then bench lines per path.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_onepass.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_onepass.log | tail -15
[ $rc -eq 0 ] || exit $rc
for cfg in "residue auto" "residue split" "residue onepass" "atom split" "atom onepass" "mixed split" "mixed onepass"; do
  set -- $cfg
  timeout -k 10 240 python bench.py --graphs $1 --ginet-path $2 --steps 40 --warmup 8 --no-cpu-baseline --no-stream-copy > gpurun_out/bench_path_$1_$2.log 2>&1; rc=$?
  echo "$1 $2 rc=$rc $(grep '^{' gpurun_out/bench_path_$1_$2.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["roofline"]["kernel_ms_avg"])')"
  ok $rc || exit $rc
done
for dt in bf16; do
  timeout -k 10 240 python bench.py --graphs atom --dtype $dt --ginet-path onepass --steps 40 --warmup 8 --no-cpu-baseline --no-stream-copy > gpurun_out/bench_atom_onepass_$dt.log 2>&1; rc=$?
  echo "atom onepass $dt rc=$rc $(grep '^{' gpurun_out/bench_atom_onepass_$dt.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["roofline"]["kernel_ms_avg"])')"
done
exit 0
