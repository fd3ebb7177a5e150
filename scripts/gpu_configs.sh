#!/bin/bash
# The other BASELINE.json configs as diagnostic bench lines (the driver's line is the default config):
# FoutNet residue (config 3), GINet atom-level (config 4 shape, 1 GPU), GINet mixed (config 5 shape), VanillaNetwork.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/bench_configs.jsonl
: > $out
for cfg in "--model foutnet --graphs residue" "--model ginet --graphs atom" "--model ginet --graphs atom --dtype bf16" "--model ginet --graphs mixed" "--model vanilla --graphs residue" "--model vanilla --graphs mixed" "--model vanilla --graphs atom" "--model foutnet --graphs mixed" "--model sgat --graphs residue" "--model sgat --graphs mixed" "--model ginet_nocluster --graphs residue" "--model ginet_nocluster --graphs mixed"; do
  echo "== $cfg"
  timeout -k 10 400 python bench.py --steps 100 --warmup 10 $cfg > gpurun_out/bench_cfg.log 2>&1; rc=$?
  grep '^{' gpurun_out/bench_cfg.log >> $out
  grep -v amdgpu.ids gpurun_out/bench_cfg.log | tail -3 | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
done
