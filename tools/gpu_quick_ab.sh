#!/bin/bash
# tests given in $TESTS, then $ROUNDS interleaved bench rounds of $CONFIG for each ";"-separated env set in $ENVS
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-qab}
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread $TESTS > $OUT/test.log 2>&1; rc=$?; tail -2 $OUT/test.log
  [ $rc -eq 0 ] || exit $rc
fi
IFS=';' read -ra SETS <<< "${ENVS:-X=1}"
for rep in $(seq 1 ${ROUNDS:-3}); do
  i=0
  for e in "${SETS[@]}"; do
    i=$((i+1))
    env $e timeout -k 10 300 python bench.py --config ${CONFIG:-cfg2} ${BENCH_ARGS} --cpu-baseline-seconds 0 > $OUT/b_${i}_$rep.log 2>&1 || exit $?
    echo "$rep [$e] $(tail -1 $OUT/b_${i}_$rep.log | cut -c90-135)"
  done
done
