#!/bin/bash
# The one GPU recipe (r06: replaces the per-round gpu_r0*.sh one-offs).
#
#   bash scripts/gpu.sh <out-subdir> <section> [section ...]
#
# Every step runs under its own `timeout -k`, and the script stops at the
# first failure (no retries).  Results go to gpurun_out/<out-subdir>/; copy
# the ones that are evidence into profiles/<round>/.
#
# sections:
#   test        pytest -m gpu (one process) + __graft_entry__.smoke()
#   test:<expr> pytest -m gpu -k <expr>
#   bench       headline line at the default step counts (CPU baseline included)
#   driver      headline line at the driver's counts (--steps 20 --warmup 5)
#   rocprof     rocprofv3 --kernel-trace --stats of the headline bench
#   stamps      per-phase stamps of ginet_graph_kernel (stamps build)
#   pmc         FETCH_SIZE / WRITE_SIZE / GRBM passes of the per-graph kernels
#               (ginet foutnet sgat ginet_nocluster vanilla) + the GINet MFMA pass
#   lds         LDS bank-conflict counters of ginet_graph_kernel
#   large       per-kernel HBM tables: GINet atom f32 / bf16 / mixed
#   vanilla     per-kernel HBM tables: Vanilla chunk pipeline atom / mixed
#   kernels:<w>,<w>  per-kernel HBM tables of any tools/pmc_run.py workloads (e.g. foutnet_atom)
#   configs     every BASELINE config line (+ the model variants), with CPU baselines
#   sweep       the GINet batch sweep (per-graph vs accumulating pass)
#   trainer     bench.py --trainer --validate (captured epochs / eval, load rate)
#   ddp1        the same on a one-rank RCCL group (Trainer(ngpu=2) code path)
#   ab:<v>,<w>  the headline bench per A/B library (tools/build_variant.sh), ABBA
#               (AB_ARGS: other bench.py arguments, e.g. "--model ginet --graphs atom"; AB_STEPS)
#   timeline    one GINet step's cross-kernel timeline (stamps build, tools/step_timeline.py)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${1:?out-subdir}; shift; mkdir -p $O
export TMPDIR=/tmp
fail() { echo "FAILED: $*"; exit 1; }
js() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d.get('roofline') or {}; c=d.get('cpu_baseline') or {}; print(round(d['value']), 'us/step', round(d['ms_per_step']*1000,2), 'pass_us', round(r.get('kernel_ms_avg',0)*1000,2), 'frac', r.get('frac'), 'traffic', r.get('traffic'), 'split', d.get('step_split_us'), 'cpu', c.get('value'), c.get('cores'))" "$1"; }
pmc_pass() {  # <dir> <workload> <steps> <counters...>
  local d=$1 w=$2 n=$3; shift 3
  mkdir -p "$(dirname $d)"
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" -f csv -d $d -o run -- python3 $R/tools/pmc_run.py $n $w > $d.log 2>&1)
}
per_kernel() {  # <workload> <steps>
  local W=$1 n=$2
  mkdir -p $O/pmc_$W
  (cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/kt_$W -o run -- python3 $R/tools/pmc_run.py $n $W > $O/kt_$W.log 2>&1) || fail "$W kernel trace"
  for set in FETCH_SIZE WRITE_SIZE; do pmc_pass $O/pmc_$W/$set $W $n $set || fail "$W $set"; done
  local f=$(find $O/kt_$W -name "*kernel_stats.csv" | head -1)
  python3 tools/pmc_per_kernel.py $O/pmc_$W "$f" $n > $O/pmc_per_kernel_$W.txt
  cut -c1-140 $O/pmc_per_kernel_$W.txt; grep alg_bytes $O/kt_$W.log
}
for S in "$@"; do
  echo "== $S"
  case $S in
    test)
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "^E |FAILED|Error" $O/pytest_gpu.log | head -30; fail pytest; }
      tail -2 $O/pytest_gpu.log
      timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; fail smoke; }
      echo smoke ok ;;
    test:*)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "${S#test:}" > $O/pytest_k.log 2>&1 || { grep -E "^E |FAILED|Error" $O/pytest_k.log | head -30; fail pytest-k; }
      grep -E "PASSED|SKIPPED" $O/pytest_k.log | cut -c1-150; tail -1 $O/pytest_k.log ;;
    bench)
      timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; fail bench; }
      js $O/bench_default.json ;;
    driver)
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver_steps.json 2> $O/bench_driver_steps.err || { tail $O/bench_driver_steps.err; fail driver; }
      js $O/bench_driver_steps.json ;;
    rocprof)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt_headline -o run -- python3 $R/bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/kt_headline.log 2>&1) || fail rocprof
      f=$(find $O/kt_headline -name "*kernel_stats.csv" | head -1); cp "$f" $O/rocprof_kernel_stats_headline.csv; cut -d, -f1-8 $O/rocprof_kernel_stats_headline.csv | head -6 ;;
    stamps)
      DR_LIB_NAME=libdeeprank2_amd_stamps.so timeout -k 10 200 python tools/stamp_profile.py 64 > $O/stamps_ginet_graph_kernel.txt 2>&1 || fail stamps
      grep -v amdgpu.ids $O/stamps_ginet_graph_kernel.txt | tail -30 ;;
    pmc)
      for M in ginet foutnet sgat ginet_nocluster vanilla; do
        case $M in ginet) K=ginet_graph_kernel ;; ginet_nocluster) K=ginet_nocluster_kernel ;; vanilla) K=vanilla_graph_kernel ;; *) K=fout_graph_kernel ;; esac
        i=0
        for set in FETCH_SIZE WRITE_SIZE GRBM_GUI_ACTIVE; do
          i=$((i+1)); pmc_pass $O/pmc_t_$M/p$i $M 40 $set || { tail -5 $O/pmc_t_$M/p$i.log; fail "$M pmc $set"; }
        done
        python3 tools/pmc_summary.py $O/pmc_t_$M $K > $O/pmc_${M}_graph_kernel.txt; cat $O/pmc_${M}_graph_kernel.txt
      done
      pmc_pass $O/pmc_m_ginet/p1 ginet 40 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CU_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT || fail "mfma pmc"
      python3 tools/pmc_summary.py $O/pmc_m_ginet ginet_graph_kernel > $O/pmc_mfma_ginet.txt; cat $O/pmc_mfma_ginet.txt ;;
    lds)
      pmc_pass $O/pmc_lds/p1 ginet 40 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || fail "lds pmc"
      python3 tools/pmc_summary.py $O/pmc_lds ginet_graph_kernel > $O/pmc_lds_ginet.txt; cat $O/pmc_lds_ginet.txt ;;
    large)
      for W in ginet_atom ginet_atom_bf16 ginet_mixed; do per_kernel $W 20; done ;;
    vanilla)
      for W in vanilla_atom vanilla_mixed; do per_kernel $W 20; done ;;
    kernels:*)  # kernels:<workload>,... : per-kernel HBM tables of any tools/pmc_run.py workloads
      IFS=, read -ra WS <<< "${S#kernels:}"; for W in "${WS[@]}"; do per_kernel $W 20; done ;;
    configs)
      : > $O/bench_configs.jsonl
      for cfg in "--model foutnet --graphs residue" "--model ginet --graphs atom" "--model ginet --graphs atom --dtype bf16" "--model ginet --graphs mixed" "--model vanilla --graphs mixed" "--model vanilla --graphs atom" "--model vanilla --graphs residue" "--model sgat --graphs residue" "--model ginet_nocluster --graphs residue"; do
        timeout -k 10 400 python bench.py --steps 100 --warmup 10 $cfg > $O/cfg.log 2>&1 || { tail -5 $O/cfg.log; fail "$cfg"; }
        grep '^{' $O/cfg.log | tail -1 >> $O/bench_configs.jsonl
        echo "$cfg | $(js $O/cfg.log)"
      done ;;
    sweep)
      : > $O/batch_sweep_ginet.jsonl
      for B in 64 256 1024 4096 16384; do
        nb=4; [ $B -ge 4096 ] && nb=2; [ $B -ge 16384 ] && nb=1
        timeout -k 10 400 python bench.py --batch $B --batches $nb --steps 20 --warmup 3 --no-cpu-baseline --no-stream-copy > $O/sweep.log 2>&1 || { tail -5 $O/sweep.log; fail "sweep B=$B"; }
        grep '^{' $O/sweep.log | tail -1 >> $O/batch_sweep_ginet.jsonl; echo "B=$B | $(js $O/sweep.log)"
      done ;;
    trainer)
      timeout -k 10 500 python bench.py --trainer --validate --batches 64 > $O/bench_trainer_b64_validate.json 2> $O/bench_trainer.err || { tail $O/bench_trainer.err; fail trainer; }
      cut -c1-600 $O/bench_trainer_b64_validate.json ;;
    ddp1)
      DR_BENCH_PG=1 timeout -k 10 500 python bench.py --trainer --validate --batches 64 > $O/bench_trainer_b64_validate_ddp1.json 2> $O/bench_trainer_ddp1.err || { tail $O/bench_trainer_ddp1.err; fail ddp1; }
      cut -c1-600 $O/bench_trainer_b64_validate_ddp1.json ;;
    ab:*)  # ab:<variant>,<variant>,... : the headline bench per library (DR_LIB_NAME; "main" = the shipped one), twice in ABBA order
      IFS=, read -ra V <<< "${S#ab:}"; order=("${V[@]}"); for ((k=${#V[@]}-1; k>=0; k--)); do order+=("${V[k]}"); done
      : > $O/ab.txt
      for v in "${order[@]}"; do
        lib=libdeeprank2_amd.so; [ "$v" = main ] || lib=libdeeprank2_amd_$v.so
        DR_LIB_NAME=$lib timeout -k 10 300 python bench.py --steps ${AB_STEPS:-200} --warmup 20 --no-cpu-baseline --no-stream-copy $AB_ARGS > $O/ab_$v.json 2> $O/ab_$v.err || { tail -5 $O/ab_$v.err; fail "ab $v"; }
        echo "$v | $(js $O/ab_$v.json)" | tee -a $O/ab.txt
      done ;;
    timeline)
      DR_LIB_NAME=libdeeprank2_amd_stamps.so timeout -k 10 200 python tools/step_timeline.py 64 20 > $O/timeline.txt 2>&1 || fail timeline
      grep -v amdgpu.ids $O/timeline.txt ;;
    *) fail "unknown section $S" ;;
  esac
done
echo done
