#!/bin/bash
# Interleaved A/B of one environment switch: VAR=name VALS="0 1" CFGS="cfg5 cfg2" ROUNDS=2 STEPS=30
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/ab_${VAR}
mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in ${CFGS:-cfg5}; do
    for v in ${VALS:-0 1}; do
      env $VAR=$v timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-30} --warmup 5 --cpu-baseline-seconds 0 > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 1; }
      echo "$c $r $VAR=$v $(grep -o '"value": [0-9.]*' $OUT/b.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $OUT/b.log)" | tee -a $OUT/summary.txt
    done
  done
done
