#!/bin/bash
# r04 end-of-round measurements (second run, after the MFMA counts pass): full GPU test suite, smoke, headline bench (driver step counts and default),
# rocprof of the headline, every BASELINE config as a diagnostic bench line, GINet large path split vs one-pass,
# and the Vanilla chunk pipeline's per-kernel HBM traffic (FETCH_SIZE / WRITE_SIZE passes).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r04g; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver_steps.json 2> $O/bench_driver_steps.err; rc=$?; echo "bench(20,5) rc=$rc"; cut -c1-300 $O/bench_driver_steps.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $O/bench_default.json 2> $O/bench_default.err; rc=$?; echo "bench(200,20) rc=$rc"; [ $rc -eq 0 ] || exit $rc
: > $O/bench_configs.jsonl
for cfg in "--model foutnet --graphs residue" "--model ginet --graphs atom" "--model ginet --graphs atom --dtype bf16" "--model ginet --graphs mixed" "--model ginet --graphs mixed --ginet-path onepass" "--model ginet --graphs atom --ginet-path onepass" "--model vanilla --graphs residue" "--model vanilla --graphs mixed" "--model vanilla --graphs atom" "--model foutnet --graphs mixed" "--model sgat --graphs residue" "--model sgat --graphs mixed" "--model ginet_nocluster --graphs residue" "--model ginet_nocluster --graphs mixed"; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 $cfg > $O/bench_cfg.log 2> $O/bench_cfg.err; rc=$?
  grep '^{' $O/bench_cfg.log >> $O/bench_configs.jsonl
  echo "== $cfg rc=$rc: $(grep '^{' $O/bench_cfg.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"])')"
  [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_headline -o run -- python3 $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/prof_headline.log 2>&1; rc=$?
echo "rocprof headline rc=$rc"; [ $rc -eq 0 ] || exit $rc
for W in vanilla_atom vanilla_mixed; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/kt_$W -o run -- python3 $R/tools/pmc_run.py 20 $W > $O/kt_$W.log 2>&1
  rc=$?; echo "$W kernel-trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
  for set in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $set -f csv -d $O/pmc_$W/$set -o run -- python3 $R/tools/pmc_run.py 20 $W > $O/pmc_${W}_$set.log 2>&1
    rc=$?; echo "$W $set rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  f=$(find $O/kt_$W -name "*kernel_stats.csv" | head -1)
  (cd $R && python3 tools/pmc_per_kernel.py $O/pmc_$W "$f" 20 > $O/pmc_per_kernel_$W.txt; head -12 $O/pmc_per_kernel_$W.txt | cut -c1-120; tail -2 $O/pmc_per_kernel_$W.txt)
done
cd $R
for W in atom mixed; do
  DR_LIB_NAME=libdeeprank2_amd_stamps.so timeout -k 10 120 python tools/vchunk_stamps.py $W > $O/stamps_vchunk_${W}.txt 2>&1; rc=$?; echo "stamps $W rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
