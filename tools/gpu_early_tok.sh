#!/bin/bash
# cfg5: where the token table's early Adam update runs (side stream after the head update / the step's own stream)
# and on how many workgroups; interleaved rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-etok}
mkdir -p $OUT
for m in 0 1; do
  RS_EARLY_TOKEN_MAIN=$m RS_EARLY_TOKEN_ADAM_WG=8192 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bert.py -k "early_head" > $OUT/test_$m.log 2>&1; rc=$?; tail -1 $OUT/test_$m.log
  [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2 3; do
  for v in "0 256" "0 8192" "1 8192" "1 2048"; do
    set -- $v
    RS_EARLY_TOKEN_MAIN=$1 RS_EARLY_TOKEN_ADAM_WG=$2 timeout -k 10 300 python bench.py --config cfg5 --steps 30 --warmup 5 --cpu-baseline-seconds 0 > $OUT/cfg5_m$1_w$2_$rep.log 2>&1 || exit $?
    echo "$rep main=$1 wg=$2 $(tail -1 $OUT/cfg5_m$1_w$2_$rep.log | cut -c90-140)"
  done
done
