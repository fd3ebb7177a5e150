#!/bin/bash
# GINet graph kernel diagnostics: phase stamps (stamps build) + PMC passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 200 python tools/stamp_profile.py 64 > gpurun_out/stamps.log 2>&1; rc=$?; echo "stamps rc=$rc"; grep -v amdgpu.ids gpurun_out/stamps.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc.sh
