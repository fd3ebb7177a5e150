#!/bin/bash
# r05 final (A): GPU suite + smoke, headline bench lines, rocprof stats and PMC of the headline at HEAD.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/r05fa; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $O/bench_default.json 2> $O/bench_default.err; rc=$?; echo "bench rc=$rc"; cut -c1-200 $O/bench_default.json; [ $rc -eq 0 ] || exit $rc
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt_headline -o run -- python3 $R/bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/kt_headline.log 2>&1); echo "headline rocprof rc=$?"
bash scripts/gpu_r05_evidence.sh r05fa/ev bench pmc_headline stamps
echo done
