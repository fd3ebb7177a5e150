#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05i; mkdir -p $O
for nr in 32 85; do
  DR_PIPED_NR=$nr DR_LIB_NAME=libdeeprank2_amd_stamps.so timeout -k 10 120 python tools/piped_stamps.py 64 30 > $O/piped_stamps_nr$nr.txt 2>&1; rc=$?
  echo "NR $nr rc=$rc"; grep -v amdgpu $O/piped_stamps_nr$nr.txt; [ $rc -eq 0 ] || exit $rc
done
