#!/bin/bash
# GPU pass: all parity tests, then bench + rocprof kernel trace for the configs in $CONFIGS.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-all}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -5 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-cfg2}; do
  timeout -k 10 600 python bench.py --config $c ${BENCH_ARGS} > $OUT/bench_$c.log 2>&1; rc=$?; tail -1 $OUT/bench_$c.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o prof -- python3 bench.py --config $c --steps 50 --warmup 10 --cpu-baseline-seconds 0 > $OUT/rocprof_$c.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { tail -20 $OUT/rocprof_$c.log; exit $rc; }
done
echo done
