#!/bin/bash
# Bench line + rocprof kernel stats of the same command (kernel-average cross-check),
# plus optional extra rocprof'd bench configurations given as arguments ("--model vanilla" ...).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 240 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/bench.log | cut -c1-1500
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
i=0
for cfg in "" "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof$i -o run -- python3 $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline $cfg > $R/gpurun_out/prof$i.log 2>&1; rc=$?
  echo "== rocprof [$cfg] rc=$rc"; grep '^{' $R/gpurun_out/prof$i.log | cut -c1-700
  f=$(find $R/gpurun_out/prof$i -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-4 "$f" | cut -c1-160 | sed -n 1,16p
  [ $rc -eq 0 ] || exit $rc
done
