cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for cfg in "--force-large 64" "--force-large 96" "--force-large 128" "--batch 256" "--batch 1024"; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline $cfg > gpurun_out/diag.log 2>&1; rc=$?
  echo "== [$cfg] rc=$rc"; grep '^{' gpurun_out/diag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_ms_avg'], r['frac'])"
  [ $rc -eq 0 ] || exit $rc
done
