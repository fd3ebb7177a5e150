#!/bin/bash
# Vanilla pipeline tiled edge kernels: parity, bench (atom B=32, mixed B=64), rocprof of the atom run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest tests/test_gpu_vanilla.py tests/test_gpu_mixed.py tests/test_gpu_ginet_nocluster.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r03/pt_vtile.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -v amdgpu.ids gpurun_out/r03/pt_vtile.log | tail -4; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/r03/bench_vtile.jsonl; : > $out
for g in atom mixed; do
  timeout -k 10 200 python bench.py --model vanilla --graphs $g --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r03/b.log 2>&1; rc=$?
  echo "$g rc=$rc: $(grep '^{' gpurun_out/r03/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  grep '^{' gpurun_out/r03/b.log >> $out
  [ $rc -eq 0 ] || { tail -5 gpurun_out/r03/b.log; exit $rc; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/r03/prof_vatom -o run -- python3 $R/bench.py --model vanilla --graphs atom --steps 50 --warmup 5 --no-cpu-baseline > $R/gpurun_out/r03/prof_vatom.log 2>&1; rc=$?
echo "rocprof rc=$rc"
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('/root/repo/gpurun_out/r03/prof_vatom/run_kernel_stats.csv')))
for r in rows[:8]:
    print(f"{r['Name'][:60]:60s} {r['Calls']:>6} {float(r['AverageNs'])/1e3:9.2f} us {r['Percentage']:>6}")
PY
exit $rc
