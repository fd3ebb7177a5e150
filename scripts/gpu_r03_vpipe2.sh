#!/bin/bash
# Vanilla pipeline iteration: parity tests, atom / mixed bench lines, rocprof kernel stats of the atom step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest tests/test_gpu_vanilla.py tests/test_gpu_vanilla_fused.py tests/test_gpu_mixed.py tests/test_gpu_ginet_nocluster.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03/pt_vpipe2.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r03/pt_vpipe2.log; [ $rc -eq 0 ] || exit $rc
for g in atom mixed; do :
  timeout -k 10 240 python bench.py --model vanilla --graphs $g --steps 60 --warmup 6 --no-cpu-baseline > gpurun_out/r03/bench_vanilla_$g.json 2> gpurun_out/r03/bench_vanilla_$g.err; rc=$?
  echo "vanilla $g rc=$rc: $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["ms_per_step"])' gpurun_out/r03/bench_vanilla_$g.json)"; [ $rc -eq 0 ] || exit $rc
done
R=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/r03/prof_vatom -o run -- python3 $R/bench.py --model vanilla --graphs atom --steps 60 --warmup 6 --no-cpu-baseline --no-stream-copy > $R/gpurun_out/r03/prof_vatom.log 2>&1; rc=$?
echo "rocprof rc=$rc"
f=$(find $R/gpurun_out/r03/prof_vatom -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-4 "$f" | cut -c1-120 | sed -n 1,14p

[ $rc -eq 0 ] || exit $rc
cd $R
timeout -k 10 240 python bench.py --model ginet --graphs atom --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r03/bench_ginet_atom.json 2> gpurun_out/r03/bench_ginet_atom.err; rc=$?
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python bench.py --model ginet_nocluster --graphs mixed --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r03/bench_nc_mixed.json 2> gpurun_out/r03/bench_nc_mixed.err; rc=$?
echo "nc mixed rc=$rc: $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_avg"])' gpurun_out/r03/bench_nc_mixed.json)"
echo "ginet atom rc=$rc: $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_avg"])' gpurun_out/r03/bench_ginet_atom.json)"
exit $rc
