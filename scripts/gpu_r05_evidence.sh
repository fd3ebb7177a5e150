#!/bin/bash
# r05 counter evidence for every BASELINE config line:
#   bash scripts/gpu_r05_evidence.sh <out-subdir> [sections...]
# sections: bench stamps floor pmc_headline pmc_large pmc_vanilla sweep (default: all)
#  - bench: headline line at the driver's step counts
#  - stamps: per-phase stamps of ginet_graph_kernel (stamps build)
#  - floor: the per-kernel launch floor inside a hipGraph (tools/launch_floor.hip)
#  - pmc_headline: FETCH_SIZE / WRITE_SIZE / GRBM passes + the MFMA pass of the
#    per-graph kernels (ginet, foutnet) -> pmc_<model>_graph_kernel.txt, pmc_mfma_ginet.txt
#  - pmc_large / pmc_vanilla: per-kernel HBM tables of the multi-kernel graph
#    passes (GINet tile + tail, atom f32 / bf16 / mixed; Vanilla chunk pipeline)
#  - sweep: the GINet batch sweep (graphs/s and the step split per B)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${1:-r05a}; shift; mkdir -p $O
SECTIONS="${@:-bench stamps floor pmc_headline pmc_large pmc_vanilla sweep}"
has() { [[ " $SECTIONS " == *" $1 "* ]]; }
export TMPDIR=/tmp
if has bench; then
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver_steps.json 2> $O/bench_driver_steps.err; rc=$?
  echo "bench(20,5) rc=$rc"; cut -c1-200 $O/bench_driver_steps.json; [ $rc -eq 0 ] || exit $rc
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print("graphs/s", d["value"], "us/step", d["ms_per_step"]*1e3, "split", d["step_split_us"])' $O/bench_driver_steps.json
fi
if has stamps; then
  DR_LIB_NAME=libdeeprank2_amd_stamps.so timeout -k 10 200 python tools/stamp_profile.py 64 > $O/stamps_ginet_graph_kernel.txt 2>&1; rc=$?
  echo "stamps rc=$rc"; grep -v amdgpu.ids $O/stamps_ginet_graph_kernel.txt; [ $rc -eq 0 ] || exit $rc
fi
if has floor; then
  hipcc --offload-arch=gfx950 -O3 tools/launch_floor.hip -o /tmp/launch_floor && timeout -k 10 120 /tmp/launch_floor > $O/launch_floor.txt 2>&1; rc=$?
  echo "launch floor rc=$rc"; cat $O/launch_floor.txt; [ $rc -eq 0 ] || exit $rc
fi
pmc_pass() {  # <dir> <workload> <steps> <counters...>
  local d=$1 w=$2 n=$3; shift 3
  mkdir -p "$(dirname $d)"
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" -f csv -d $d -o run -- python3 $R/tools/pmc_run.py $n $w > $d.log 2>&1)
}
if has pmc_headline; then
  for M in ginet foutnet; do
    case $M in ginet) K=ginet_graph_kernel ;; *) K=fout_graph_kernel ;; esac
    i=0
    for set in FETCH_SIZE WRITE_SIZE GRBM_GUI_ACTIVE; do
      i=$((i+1)); pmc_pass $O/pmc_t_$M/p$i $M 40 $set; rc=$?; echo "$M pass $i ($set) rc=$rc"
      [ $rc -eq 0 ] || { tail -5 $O/pmc_t_$M/p$i.log; exit $rc; }
    done
    python3 tools/pmc_summary.py $O/pmc_t_$M $K > $O/pmc_${M}_graph_kernel.txt; cat $O/pmc_${M}_graph_kernel.txt; grep alg_bytes $O/pmc_t_$M/p1.log
  done
  pmc_pass $O/pmc_m_ginet/p1 ginet 40 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CU_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT; rc=$?
  echo "ginet mfma pass rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 tools/pmc_summary.py $O/pmc_m_ginet ginet_graph_kernel > $O/pmc_mfma_ginet.txt; cat $O/pmc_mfma_ginet.txt
fi
per_kernel() {  # <workload> <steps>
  local W=$1 n=$2
  mkdir -p $O/pmc_$W
  (cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/kt_$W -o run -- python3 $R/tools/pmc_run.py $n $W > $O/kt_$W.log 2>&1); rc=$?
  echo "$W kernel-trace rc=$rc"; [ $rc -eq 0 ] || return $rc
  for set in FETCH_SIZE WRITE_SIZE; do
    pmc_pass $O/pmc_$W/$set $W $n $set; rc=$?; echo "$W $set rc=$rc"; [ $rc -eq 0 ] || return $rc
  done
  f=$(find $O/kt_$W -name "*kernel_stats.csv" | head -1)
  python3 tools/pmc_per_kernel.py $O/pmc_$W "$f" $n > $O/pmc_per_kernel_$W.txt; cut -c1-120 $O/pmc_per_kernel_$W.txt | head -8; tail -2 $O/pmc_per_kernel_$W.txt
  grep alg_bytes $O/kt_$W.log
}
if has pmc_large; then
  for W in ginet_atom ginet_atom_bf16 ginet_mixed; do per_kernel $W 20 || exit $?; done
fi
if has pmc_vanilla; then
  for W in vanilla_atom vanilla_mixed; do per_kernel $W 20 || exit $?; done
fi
if has sweep; then
  : > $O/batch_sweep_ginet.jsonl
  for B in 64 256 1024 4096 16384; do
    nb=4; [ $B -ge 4096 ] && nb=2; [ $B -ge 16384 ] && nb=1
    timeout -k 10 400 python bench.py --batch $B --batches $nb --steps 20 --warmup 3 --no-cpu-baseline --no-stream-copy > $O/sweep.log 2>&1; rc=$?
    echo "== B=$B rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/sweep.log; exit $rc; }
    grep '^{' $O/sweep.log | tee -a $O/batch_sweep_ginet.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_ms_avg'], r['frac'], d['step_split_us'])"
  done
fi
echo done
