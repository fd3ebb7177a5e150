#!/bin/bash
# r05: accumulating pass with scalar y / once-per-launch step counter, M0 saved around the asm DMA.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05o; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_acc_pass.py tests/test_gpu_trainer.py tests/test_gpu_train_step.py tests/test_gpu_ginet.py > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest.log | head -20; exit $rc; }
DR_ACC_PREFETCH=1 timeout -k 10 300 python tools/acc_stamps.py 4096 > $O/stamps_pf.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/stamps_pf.txt
for B in 4096 16384; do
  nb=2; [ $B -ge 16384 ] && nb=1
  timeout -k 10 400 python bench.py --batch $B --batches $nb --steps 20 --warmup 3 --no-cpu-baseline --no-stream-copy > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  echo "B=$B $(grep '^{' $O/b.log | tee -a $O/sweep.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d.get('step_split_us') or {}; print(round(d['value']), 'step_us', round(d['ms_per_step']*1000,2), 'pass_us', s.get('graph_pass'), 'reduce_us', s.get('reduce_adam'))")"
done
