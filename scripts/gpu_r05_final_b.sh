#!/bin/bash
# r05 final (B): the other config lines, the accumulating-pass sweep, the trainer line at HEAD.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05fb; mkdir -p $O
: > $O/bench_configs.jsonl
for cfg in "--model foutnet --graphs residue" "--model ginet --graphs atom" "--model ginet --graphs atom --dtype bf16" "--model ginet --graphs mixed" "--model vanilla --graphs residue" "--model vanilla --graphs mixed" "--model vanilla --graphs atom" "--model sgat --graphs residue" "--model ginet_nocluster --graphs residue"; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline $cfg > $O/cfg.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "$cfg rc=$rc"; tail -5 $O/cfg.log; exit $rc; }
  echo "$cfg | $(grep '^{' $O/cfg.log | tee -a $O/bench_configs.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['value']), 'us/step', round(d['ms_per_step']*1000,1), 'pass', round(r['kernel_ms_avg']*1000,1), 'frac', round(r['frac'],4), 'traffic', r.get('traffic'))")"
done
: > $O/sweep.jsonl
for B in 1024 4096 16384; do
  nb=4; [ $B -ge 4096 ] && nb=2; [ $B -ge 16384 ] && nb=1
  for mode in "--acc off" "--acc on"; do
    timeout -k 10 400 python bench.py --batch $B --batches $nb --steps 20 --warmup 3 --no-cpu-baseline --no-stream-copy $mode > $O/sweep.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { tail -5 $O/sweep.log; exit $rc; }
    echo "B=$B $mode | $(grep '^{' $O/sweep.log | tee -a $O/sweep.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d.get('step_split_us') or {}; print(round(d['value']), 'step_us', round(d['ms_per_step']*1000,2), 'pass_us', s.get('graph_pass'), 'reduce_us', s.get('reduce_adam'))")" | tee -a $O/sweep.txt
  done
done
timeout -k 10 400 python bench.py --trainer --validate --batches 64 > $O/bench_trainer_b64_validate.json 2> $O/bench_trainer.err; rc=$?; echo "trainer rc=$rc"; cut -c1-300 $O/bench_trainer_b64_validate.json
echo done
