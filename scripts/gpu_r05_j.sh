#!/bin/bash
# r05 HEAD: GPU suite, smoke, headline + trainer benches, then counter evidence.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05j; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver_steps.json 2> $O/bench_driver_steps.err; rc=$?; echo "bench(20,5) rc=$rc"; cut -c1-240 $O/bench_driver_steps.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $O/bench_default.json 2> $O/bench_default.err; rc=$?; echo "bench(200,20) rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --trainer --validate --batches 64 > $O/bench_trainer_b64.json 2> $O/bench_trainer.err; rc=$?; echo "trainer rc=$rc"; cut -c1-400 $O/bench_trainer_b64.json; [ $rc -eq 0 ] || { tail -5 $O/bench_trainer.err; exit $rc; }
DR_BENCH_PG=1 timeout -k 10 400 python bench.py --trainer --validate --batches 64 > $O/bench_trainer_b64_ddp.json 2> $O/bench_trainer_ddp.err; rc=$?; echo "trainer ddp rc=$rc"; cut -c1-400 $O/bench_trainer_b64_ddp.json; [ $rc -eq 0 ] || { tail -5 $O/bench_trainer_ddp.err; exit $rc; }
bash scripts/gpu_r05_evidence.sh r05j/ev stamps pmc_headline pmc_large pmc_vanilla sweep
