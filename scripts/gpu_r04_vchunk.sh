#!/bin/bash
# Vanilla chunk-fused pipeline: parity tests, atom / mixed bench lines (chunk-fused vs 16-row tiles), kernel stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_vanilla.py tests/test_gpu_vanilla_fused.py tests/test_gpu_mixed.py tests/test_gpu_foutnet.py tests/test_gpu_sgat.py tests/test_gpu_trainer.py tests/test_gpu_distributed.py -x -v --timeout 120 --timeout-method thread > $O/pt_vchunk.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error|error" $O/pt_vchunk.log | tail -8; [ $rc -eq 0 ] || exit $rc
for g in atom mixed; do
  for T in 64 16; do
    DR_VANILLA_TILE=$T timeout -k 10 240 python bench.py --model vanilla --graphs $g --steps 60 --warmup 6 --no-cpu-baseline --no-stream-copy > $O/bench_vanilla_${g}_t$T.json 2> $O/bench_vanilla_${g}_t$T.err; rc=$?
    echo "vanilla $g tile $T rc=$rc: $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["ms_per_step"], d["final_loss"])' $O/bench_vanilla_${g}_t$T.json)"; [ $rc -eq 0 ] || exit $rc
  done
done
R=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $R/$O/prof_vchunk_atom -o run -- python3 $R/bench.py --model vanilla --graphs atom --steps 60 --warmup 6 --no-cpu-baseline --no-stream-copy > $R/$O/prof_vchunk_atom.log 2>&1; rc=$?
echo "rocprof rc=$rc"
f=$(find $R/$O/prof_vchunk_atom -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-4 "$f" | cut -c1-110 | sed -n 1,14p
[ $rc -eq 0 ] || exit $rc
cd $R
timeout -k 10 300 python bench.py --trainer --epochs 3 --batches 16 > $O/bench_trainer.json 2> $O/bench_trainer.err; rc=$?
echo "trainer rc=$rc"; cat $O/bench_trainer.json | cut -c1-600; [ $rc -eq 0 ] || { tail -20 $O/bench_trainer.err; exit $rc; }
