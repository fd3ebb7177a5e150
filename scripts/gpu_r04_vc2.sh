#!/bin/bash
# Vanilla chunk kernels with batched prologues: parity, atom / mixed bench lines, phase stamps, kernel stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r04; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_vanilla.py tests/test_gpu_vanilla_fused.py tests/test_gpu_mixed.py -x -v --timeout 120 --timeout-method thread > $O/pt_vc2.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error" $O/pt_vc2.log | tail -6; [ $rc -eq 0 ] || exit $rc
for g in atom mixed; do
  timeout -k 10 240 python bench.py --model vanilla --graphs $g --steps 60 --warmup 6 --no-cpu-baseline --no-stream-copy > $O/bench_vc2_$g.json 2> $O/bench_vc2_$g.err; rc=$?
  echo "vanilla $g rc=$rc: $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["ms_per_step"], d["final_loss"], d.get("step_split_us"))' $O/bench_vc2_$g.json)"; [ $rc -eq 0 ] || exit $rc
done
DR_LIB_NAME=libdeeprank2_amd_stamps.so timeout -k 10 120 python tools/vchunk_stamps.py atom > $O/vc2_stamps_atom.txt 2>&1; rc=$?
echo "stamps rc=$rc"; grep -v amdgpu.ids $O/vc2_stamps_atom.txt | cut -c1-400; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_vc2_atom -o run -- python3 $R/bench.py --model vanilla --graphs atom --steps 60 --warmup 6 --no-cpu-baseline --no-stream-copy > $O/prof_vc2_atom.log 2>&1; rc=$?
echo "rocprof rc=$rc"
f=$(find $O/prof_vc2_atom -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-4 "$f" | cut -c1-110 | sed -n 1,12p
exit $rc
