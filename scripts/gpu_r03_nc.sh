#!/bin/bash
# ginet_nocluster large-graph pipeline: parity, mixed bench line, rocprof.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest tests/test_gpu_ginet_nocluster.py tests/test_gpu_layered.py -q --timeout 120 --timeout-method thread > gpurun_out/r03/pt_nc.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -v amdgpu.ids gpurun_out/r03/pt_nc.log | tail -40
[ $rc -eq 0 ] || exit $rc
out=gpurun_out/r03/bench_nc.jsonl; : > $out
for g in mixed atom residue; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 5 --model ginet_nocluster --graphs $g --no-cpu-baseline > gpurun_out/r03/b.log 2>&1; rc=$?
  echo "$g rc=$rc: $(grep '^{' gpurun_out/r03/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  grep '^{' gpurun_out/r03/b.log >> $out
  [ $rc -eq 0 ] || { tail -5 gpurun_out/r03/b.log; exit $rc; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/r03/prof_ncmixed -o run -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline --model ginet_nocluster --graphs mixed > $R/gpurun_out/r03/prof_nc.log 2>&1; rc=$?
echo "rocprof rc=$rc"
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('/root/repo/gpurun_out/r03/prof_ncmixed/run_kernel_stats.csv')))
for r in rows[:10]:
    print(f"{r['Name'][:60]:60s} {r['Calls']:>6} {float(r['AverageNs'])/1e3:9.1f} us {r['Percentage']:>6}")
PY
exit $rc
