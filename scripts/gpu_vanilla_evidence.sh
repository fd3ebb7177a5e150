#!/bin/bash
# Vanilla split evidence: rocprof kernel stats of the residue bench, then every config bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_van -o van -- python3 bench.py --model vanilla --graphs residue --steps 50 --warmup 10 --no-cpu-baseline --no-stream-copy > gpurun_out/prof_van.log 2>&1; rc=$?
echo "rocprof rc=$rc"; find gpurun_out/prof_van -name "*kernel_stats.csv" | head -3
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_configs.sh
