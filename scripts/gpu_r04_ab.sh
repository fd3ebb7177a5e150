#!/bin/bash
# A/B of a library change on the same box: libdeeprank2_amd_prev.so (before) vs libdeeprank2_amd.so (after),
# interleaved bench lines, then GPU tests on the new library.
#   bash scripts/gpu_r04_ab.sh "<cfg>;<cfg>;..." "<pytest -k expression>" [reps]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/ab; mkdir -p $O
IFS=';' read -ra CFGS <<< "$1"
K="$2"; REPS=${3:-2}
: > $O/ab.txt
for rep in $(seq 1 $REPS); do
for cfg in "${CFGS[@]}"; do
  LIBS="libdeeprank2_amd_prev.so libdeeprank2_amd.so"; [ $((rep % 2)) -eq 0 ] && LIBS="libdeeprank2_amd.so libdeeprank2_amd_prev.so"  # ABBA
  for lib in $LIBS; do
    DR_LIB_NAME=$lib timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline $cfg > $O/b.log 2> $O/b.err; rc=$?
    echo "$lib $cfg rc=$rc: $(grep '^{' $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1000,1), round(d["roofline"]["kernel_ms_avg"]*1000,2), d.get("step_split_us"))')" | tee -a $O/ab.txt
    [ $rc -eq 0 ] || { tail -5 $O/b.err; exit $rc; }
  done
done
done
# per-kernel averages of both libraries (rocprof kernel trace of tools/pmc_run.py) for the workloads in $PROF
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  for W in ${PROF//,/ }; do
    for lib in libdeeprank2_amd_prev.so libdeeprank2_amd.so; do
      DR_LIB_NAME=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/kt_${W}_$lib -o run -- python3 $R/tools/pmc_run.py 20 $W > $O/kt.log 2>&1; rc=$?
      [ $rc -eq 0 ] || { echo "rocprof $W $lib rc=$rc"; tail -5 $O/kt.log; exit $rc; }
      f=$(find $O/kt_${W}_$lib -name "*kernel_stats.csv" | head -1)
      echo "== $W $lib"; python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    n=r['Name']
    if any(k in n for k in ('vc_','vb_head','reduce_adam','ginet','fout','large','conv','tail')): print('  %-40s %6s calls %8.2f us' % (n[:40], r['Calls'], float(r['AverageNs'])/1e3))
" $f | tee -a $O/ab.txt
    done
  done
  cd $R
fi
[ -n "$K" ] || exit 0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log; exit $rc
