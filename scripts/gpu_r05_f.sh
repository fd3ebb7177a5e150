#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/gpu_pmc_icache.sh r05f/pmc "base - pf" || exit $?
bash scripts/gpu_ab.sh r05f/ab "base - pf shfl onlycl1" "--model ginet" 2 || exit $?
