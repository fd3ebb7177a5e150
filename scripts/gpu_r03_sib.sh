#!/bin/bash
# GINet sibling split: parity, bench for k = 1..4 (driver step counts), rocprof of k=4.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_ginet.py tests/test_gpu_train_step.py -q --timeout 120 --timeout-method thread > gpurun_out/r03/pt_sib.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -v amdgpu.ids gpurun_out/r03/pt_sib.log | tail -30
[ $rc -eq 0 ] || exit $rc
out=gpurun_out/r03/bench_sib.jsonl; : > $out
for k in 1 2 3 4 1 4; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --sibling-split $k --no-cpu-baseline > gpurun_out/r03/b.log 2>&1; rc=$?
  echo "k=$k rc=$rc: $(grep '^{' gpurun_out/r03/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["roofline"]["kernel_ms_avg"])')"
  grep '^{' gpurun_out/r03/b.log | sed "s/^{/{\"sibling_split\": $k, /" >> $out
  [ $rc -eq 0 ] || { tail -5 gpurun_out/r03/b.log; exit $rc; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/r03/prof_sib -o run -- python3 $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline --sibling-split 4 > $R/gpurun_out/r03/prof_sib.log 2>&1; rc=$?
echo "rocprof rc=$rc"
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('/root/repo/gpurun_out/r03/prof_sib/run_kernel_stats.csv')))
for r in rows[:6]:
    print(f"{r['Name'][:60]:60s} {r['Calls']:>6} {float(r['AverageNs'])/1e3:9.2f} us {r['Percentage']:>6}")
PY
exit $rc
