#!/bin/bash
# r05: accumulating pass with the idle-wave prefetch — parity, stamps, sweep on/off.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05acc4; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_acc_pass.py > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest.log | head; exit $rc; }
DR_ACC_PREFETCH=1 timeout -k 10 300 python tools/acc_stamps.py 4096 > $O/stamps_pf.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/stamps_pf.txt
: > $O/sweep.jsonl
for B in 1024 4096 16384; do
  nb=4; [ $B -ge 4096 ] && nb=2; [ $B -ge 16384 ] && nb=1
  for pf in "" "--acc-prefetch"; do
    timeout -k 10 400 python bench.py --batch $B --batches $nb --steps 20 --warmup 3 --no-cpu-baseline --no-stream-copy --acc on $pf > $O/sweep.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { tail -5 $O/sweep.log; exit $rc; }
    echo "B=$B $pf $(grep '^{' $O/sweep.log | tee -a $O/sweep.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d.get('step_split_us') or {}; print(round(d['value']), 'step_us', round(d['ms_per_step']*1000,2), 'pass_us', s.get('graph_pass'), 'reduce_us', s.get('reduce_adam'))")"
  done
done
echo done
