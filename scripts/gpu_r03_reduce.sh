#!/bin/bash
# Reduce kernel change: parity (one-launch bit identity, Vanilla split), benches, rocprof of the Vanilla run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out/r03
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_step.py tests/test_gpu_vanilla_fused.py tests/test_gpu_distributed.py tests/test_gpu_ginet.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r03/pt_red.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -v amdgpu.ids gpurun_out/r03/pt_red.log | tail -3; [ $rc -eq 0 ] || exit $rc
for m in vanilla vanilla ginet; do
  timeout -k 10 200 python bench.py --model $m --graphs residue --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r03/b.log 2>&1; rc=$?
  echo "$m rc=$rc: $(grep '^{' gpurun_out/r03/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["roofline"]["kernel_ms_avg"])')"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/r03/b.log; exit $rc; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/r03/prof_vres -o run -- python3 $R/bench.py --model vanilla --steps 50 --warmup 5 --no-cpu-baseline > $R/gpurun_out/r03/prof_vres.log 2>&1; rc=$?
echo "rocprof rc=$rc"
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('/root/repo/gpurun_out/r03/prof_vres/run_kernel_stats.csv')))
for r in rows[:5]:
    print(f"{r['Name'][:60]:60s} {r['Calls']:>6} {float(r['AverageNs'])/1e3:9.2f} us")
PY
exit $rc
