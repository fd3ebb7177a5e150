#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/gpu_vanilla_iter.sh || exit $?
bash scripts/gpu_ginet_iter.sh
