#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 100 python scripts/dbg_f40.py || exit 1
bash scripts/gpu_ab.sh r05q/ab "base nokeys -" "--model ginet" 3 "acc or ginet"
