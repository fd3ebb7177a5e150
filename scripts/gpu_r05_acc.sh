#!/bin/bash
# r05: accumulating GINet pass — parity tests, then the batch sweep with the
# accumulating pass on / off (auto = on past the CU count).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05acc; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_acc_pass.py tests/test_gpu_train_step.py > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
: > $O/sweep.jsonl
for B in 512 1024 4096 16384; do
  nb=4; [ $B -ge 4096 ] && nb=2; [ $B -ge 16384 ] && nb=1
  for acc in off on; do
    timeout -k 10 400 python bench.py --batch $B --batches $nb --steps 20 --warmup 3 --no-cpu-baseline --no-stream-copy --acc $acc > $O/sweep.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { tail -5 $O/sweep.log; exit $rc; }
    echo "B=$B acc=$acc $(grep '^{' $O/sweep.log | tee -a $O/sweep.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['value']), 'step_ms', round(d['ms_per_step'],4), 'pass_ms', round(r['kernel_ms_avg'],4), 'frac', round(r['frac'],3), d.get('step_split_us'))")"
  done
done
echo done
