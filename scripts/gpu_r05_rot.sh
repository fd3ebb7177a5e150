#!/bin/bash
# r05: DMA start-wave rotation in the GINet staging — stamps (B=64) and the headline A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05rot; mkdir -p $O
for v in stamps0 stamps; do
  DR_LIB_NAME=libdeeprank2_amd_$v.so timeout -k 10 200 python tools/stamp_profile.py 64 > $O/stamps_$v.txt 2>&1 || exit 1
  echo "== $v"; grep -v amdgpu.ids $O/stamps_$v.txt | head -8
done
bash scripts/gpu_ab.sh r05rot/ab "rot0 -" "--model ginet" 3 "acc or train_step or test_gpu_ginet"
timeout -k 10 300 python tools/acc_stamps.py 4096 > $O/acc_stamps.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/acc_stamps.txt
bash scripts/gpu_r05_acc2.sh
