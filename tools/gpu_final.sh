#!/bin/bash
# final check: GPU suite + smoke, then the driver-shaped bench (steps 20, warmup 5) with / without graph upload
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-final}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -2 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "__import__('__graft_entry__').smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -2 $OUT/smoke.log
for r in 1 2 3 4; do
  for u in 0 1; do
    RS_GRAPH_UPLOAD=$u timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/drv_u${u}_$r.log 2>&1 || exit $?
    echo "$r upload=$u $(tail -1 $OUT/drv_u${u}_$r.log | cut -c90-135)"
  done
done
