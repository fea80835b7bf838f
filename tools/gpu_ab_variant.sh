#!/bin/bash
# Interleaved A/B of a variant library build against the default: V=name (librecsys_hip.$V.so, tools/build_variant.sh)
# CFGS="cfg3 cfg5" ROUNDS=2 STEPS=30
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/abv_$V
mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in ${CFGS:-cfg3}; do
    for v in default $V; do
      if [ $v = default ]; then unset RS_LIB_VARIANT; else export RS_LIB_VARIANT=$v; fi
      timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-30} --warmup 5 --cpu-baseline-seconds 0 > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 1; }
      echo "$c $r $v $(grep -o '"value": [0-9.]*' $OUT/b.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $OUT/b.log) $(grep -o '"avg_launch_us": [0-9.]*' $OUT/b.log)" | tee -a $OUT/summary.txt
    done
  done
done
unset RS_LIB_VARIANT
