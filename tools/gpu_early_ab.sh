#!/bin/bash
# cfg5: the early out.weight Adam's workgroup cap (RS_EARLY_HEAD_ADAM_WG) and the end-of-step form, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-early}
mkdir -p $OUT
for rep in 1 2; do
  for wg in 0 128 256 512 1024; do
    if [ $wg = 0 ]; then E="RS_EARLY_HEAD_ADAM=0"; else E="RS_EARLY_HEAD_ADAM_WG=$wg"; fi
    env $E timeout -k 10 300 python bench.py --config cfg5 --steps 30 --warmup 5 --cpu-baseline-seconds 0 > $OUT/cfg5_${wg}_$rep.log 2>&1 || exit $?
    echo "$rep wg=$wg $(tail -1 $OUT/cfg5_${wg}_$rep.log | cut -c90-140)"
  done
done
