#!/bin/bash
# cfg5: round-4 tree (_ab/r04, built from e1fc989) against HEAD, interleaved on one box.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ab_r04
mkdir -p $OUT
for r in 1 2; do
  for t in r04 head; do
    if [ $t = r04 ]; then D=_ab/r04; else D=.; fi
    (cd $D && timeout -k 10 300 python bench.py --config ${CFG:-cfg5} --cpu-baseline-seconds 0 --steps ${STEPS:-30} --warmup 5) > $OUT/${t}_$r.log 2>&1 || { tail -5 $OUT/${t}_$r.log; exit 1; }
    echo "$t $r $(tail -1 $OUT/${t}_$r.log | cut -c1-120)"
  done
done
