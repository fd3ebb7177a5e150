#!/bin/bash
# A/B/C... of native-library variants on one box, interleaved (rotating order per rep):
#   bash scripts/gpu_ab.sh <out-subdir> "<lib suffix list>" "<cfg>;<cfg>;..." [reps] [pytest -k expr]
# suffix "-" is the regular libdeeprank2_amd.so; "x" is libdeeprank2_amd_x.so.
# Optional: a pytest -k expression run first on the regular library.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); O=$R/gpurun_out/${1:-ab}; mkdir -p $O
read -ra VARS <<< "$2"
IFS=';' read -ra CFGS <<< "$3"
REPS=${4:-2}; K="$5"
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > $O/pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
: > $O/ab.txt
n=${#VARS[@]}
for rep in $(seq 1 $REPS); do
  for cfg in "${CFGS[@]}"; do
    for j in $(seq 0 $((n - 1))); do
      v=${VARS[$(( (j + rep - 1) % n ))]}
      lib=libdeeprank2_amd.so; [ "$v" != "-" ] && lib=libdeeprank2_amd_$v.so
      DR_LIB_NAME=$lib timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-stream-copy $cfg > $O/b.log 2> $O/b.err; rc=$?
      [ $rc -eq 0 ] || { echo "$v $cfg rc=$rc"; tail -5 $O/b.err; exit $rc; }
      echo "$v | $cfg | $(grep '^{' $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("step_us", round(d["ms_per_step"]*1000,2), "pass_us", round(d["roofline"]["kernel_ms_avg"]*1000,2), "split", d.get("step_split_us") and {k: v for k, v in d["step_split_us"].items() if k != "note"})')" | tee -a $O/ab.txt
    done
  done
done
echo done
