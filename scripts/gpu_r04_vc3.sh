#!/bin/bash
# Vanilla chunk pipeline + trainer epoch capture: parity, bench lines, trainer bench, kernel stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r04; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_vanilla.py tests/test_gpu_vanilla_fused.py tests/test_gpu_mixed.py tests/test_gpu_trainer.py -x -v --timeout 120 --timeout-method thread > $O/pt_vc3.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error" $O/pt_vc3.log | tail -6; [ $rc -eq 0 ] || exit $rc
for g in atom mixed; do
  timeout -k 10 240 python bench.py --model vanilla --graphs $g --steps 60 --warmup 6 --no-cpu-baseline --no-stream-copy > $O/bench_vc3_$g.json 2> $O/bench_vc3_$g.err; rc=$?
  echo "vanilla $g rc=$rc: $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["ms_per_step"], d["final_loss"], d.get("step_split_us"))' $O/bench_vc3_$g.json | cut -c1-200)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 240 python bench.py --steps 400 --warmup 20 --no-cpu-baseline > $O/bench_vc3_ginet.json 2> $O/bench_vc3_ginet.err; rc=$?
echo "ginet rc=$rc: $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["ms_per_step"], d.get("step_split_us"))' $O/bench_vc3_ginet.json | cut -c1-200)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --trainer --epochs 3 --batches 64 > $O/bench_trainer_b64.json 2> $O/bench_trainer_b64.err; rc=$?
echo "trainer rc=$rc"; cut -c1-700 $O/bench_trainer_b64.json; [ $rc -eq 0 ] || { tail -20 $O/bench_trainer_b64.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_vc3_atom -o run -- python3 $R/bench.py --model vanilla --graphs atom --steps 60 --warmup 6 --no-cpu-baseline --no-stream-copy > $O/prof_vc3_atom.log 2>&1; rc=$?
echo "rocprof rc=$rc"
f=$(find $O/prof_vc3_atom -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-4 "$f" | cut -c1-110 | sed -n 1,12p
exit $rc
