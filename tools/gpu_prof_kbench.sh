#!/bin/bash
# tests + kernel micro-bench under rocprof (device times) + bench (cfg2 default)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pk}
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -4 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for c in ${KCONFIGS:-cfg2}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kb_$c -o kb -- python3 tools/kbench.py --config $c --reps 20 > $OUT/kb_$c.log 2>&1 || exit 1
done
for c in ${CONFIGS:-cfg2}; do
  timeout -k 10 600 python bench.py --config $c --cpu-baseline-seconds 0 > $OUT/bench_$c.log 2>&1 || { tail -20 $OUT/bench_$c.log; exit 1; }
  tail -1 $OUT/bench_$c.log | cut -c1-200
done
