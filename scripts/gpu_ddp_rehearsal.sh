#!/bin/bash
# One-GPU rehearsal of the N>1 bench path: torch.distributed.run with one rank
# and DR_BENCH_PG=1 (RCCL process group, data-parallel step with its all-reduce),
# captured (default) and eager, beside the plain N=1 line.  Same seeds, so the
# final losses must agree.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/ddp_rehearsal.jsonl
run() {
  local tag=$1; shift
  timeout -k 10 240 "$@" > gpurun_out/ddp_$tag.log 2>&1; local rc=$?
  echo "== $tag rc=$rc"; grep '^{' gpurun_out/ddp_$tag.log | tee -a gpurun_out/ddp_rehearsal.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['launch'], d['final_loss'])"
  [ $rc -eq 0 ] || { tail -30 gpurun_out/ddp_$tag.log; exit $rc; }
}
run plain python bench.py --steps 200 --warmup 20 --no-cpu-baseline
run pg_captured env DR_BENCH_PG=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --steps 200 --warmup 20
run pg_eager env DR_BENCH_PG=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29534 bench.py --steps 200 --warmup 20 --eager-ddp
