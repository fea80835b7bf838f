#!/bin/bash
# Quick GPU pass: parity tests, kernel micro-bench, short bench. Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-quick}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -15 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/kbench.py ${KB_ARGS} > $OUT/kbench.log 2>&1; rc=$?; cat $OUT/kbench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 ${BENCH_ARGS} > $OUT/bench.log 2>&1; rc=$?; tail -1 $OUT/bench.log
exit $rc
