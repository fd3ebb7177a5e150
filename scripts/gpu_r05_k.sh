#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/gpu_ab.sh r05k/ab "prev - gpipe" "--model ginet" 3 || exit $?
O=gpurun_out/r05k; : > $O/vanilla_residue.txt
for cfg in "--model vanilla --graphs residue" "--model vanilla --graphs residue --vanilla-pipeline"; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-stream-copy $cfg > $O/v.log 2> $O/v.err; rc=$?
  [ $rc -eq 0 ] || { tail -5 $O/v.err; exit $rc; }
  echo "$cfg | $(grep '^{' $O/v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("step_us", round(d["ms_per_step"]*1000,2), "pass_us", round(d["roofline"]["kernel_ms_avg"]*1000,2), d.get("step_split_us") and {k: v for k, v in d["step_split_us"].items() if k != "note"})')" | tee -a $O/vanilla_residue.txt
done
