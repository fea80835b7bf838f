#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprof kernel stats.  Every GPU step
# has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-run}
mkdir -p $OUT
echo "== pytest -m gpu" && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -5 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -2 $OUT/smoke.log && \
echo "== bench" && timeout -k 10 600 python bench.py ${BENCH_ARGS} > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log && \
echo "== rocprof" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o prof -- python3 bench.py --steps 50 --warmup 10 --cpu-baseline-seconds 0 ${BENCH_ARGS} > $OUT/rocprof.log 2>&1 && \
echo done
