#!/bin/bash
# Grouped weight gradients: 256 x 256 tiles (default) against 128 x 128 (RS_WGRAD_T256=0): tests, kernel micro-bench,
# interleaved cfg3 bench rounds.  TAG=x bash tools/gpu_wgrad_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-wgab}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_wgrad_gpu.py tests/test_bert.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for f in 0 1; do
    RS_WGRAD_T256=$f timeout -k 10 300 python bench.py --config cfg3 --cpu-baseline-seconds 0 > $OUT/cfg3_${f}_$r.log 2>&1 || { tail -5 $OUT/cfg3_${f}_$r.log; exit 1; }
    echo "T256=$f round $r: $(tail -1 $OUT/cfg3_${f}_$r.log | cut -c80-175)"
  done
done
