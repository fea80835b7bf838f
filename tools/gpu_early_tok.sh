#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-etok}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bert.py -k "early_head or overwritten" > $OUT/test.log 2>&1; rc=$?; tail -3 $OUT/test.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for f in 0 1; do
    RS_EARLY_TOKEN_ADAM=$f timeout -k 10 300 python bench.py --config cfg5 --steps 30 --warmup 5 --cpu-baseline-seconds 0 > $OUT/cfg5_tok${f}_$rep.log 2>&1 || exit $?
    echo "$rep cfg5 tok=$f $(tail -1 $OUT/cfg5_tok${f}_$rep.log | cut -c90-140)"
  done
  for f in 0 1; do
    RS_EARLY_HEAD_ADAM_SMALL=$f RS_EARLY_TOKEN_ADAM=$f timeout -k 10 300 python bench.py --config cfg3 --cpu-baseline-seconds 0 > $OUT/cfg3_small${f}_$rep.log 2>&1 || exit $?
    echo "$rep cfg3 small+tok=$f $(tail -1 $OUT/cfg3_small${f}_$rep.log | cut -c90-140)"
  done
done
