cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r03/prof_vm
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03/prof_vm -o run -- python3 bench.py --model vanilla --graphs residue --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r03/prof_vm.log 2>&1; rc=$?
echo rc=$rc; find gpurun_out/r03/prof_vm -name "*stats*" | head
