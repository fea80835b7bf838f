#!/bin/bash
# Build-free GPU pass for a kernel change: phase stamps, the named parity tests, the cfg2 bench (driver shape and
# default).  TAG=x TESTS="tests/a.py tests/b.py" bash tools/gpu_ab_quick.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-abq}
mkdir -p $OUT
if [ -x tools/micro/rowchain_phase ]; then
  timeout -k 10 60 ./tools/micro/rowchain_phase 25600 > $OUT/rowchain_phase.txt 2>&1 || { cat $OUT/rowchain_phase.txt; exit 1; }
  cat $OUT/rowchain_phase.txt
fi
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
  tail -5 $OUT/pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
for c in ${CONFIGS:-cfg2}; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --cpu-baseline-seconds 0 > $OUT/bench20_$c.log 2>&1 || { tail -20 $OUT/bench20_$c.log; exit 1; }
  tail -1 $OUT/bench20_$c.log | cut -c1-240
  timeout -k 10 300 python bench.py --config $c --cpu-baseline-seconds 0 > $OUT/bench_$c.log 2>&1 || { tail -20 $OUT/bench_$c.log; exit 1; }
  tail -1 $OUT/bench_$c.log | cut -c1-240
done
