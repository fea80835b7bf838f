#!/bin/bash
# cfg5 / cfg3: the grouped weight gradients at 128-wide tiles while the token table's update runs beside them
# (default) against no early token update; tests of the touched paths first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c5
timeout -k 10 900 python -u -m pytest tests/test_wgrad_gpu.py tests/test_bert.py tests/test_adam_gpu.py tests/test_unrolled_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/c5/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/c5/pytest.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for e in "RS_AB=1" "RS_EARLY_TOKEN_ADAM=0"; do
    env $e timeout -k 10 300 python bench.py --config cfg5 --steps 30 --warmup 5 --cpu-baseline-seconds 0 > gpurun_out/c5/b.log 2>&1 || { tail -5 gpurun_out/c5/b.log; exit 1; }
    echo "cfg5 $r $e $(grep -o '"value": [0-9.]*' gpurun_out/c5/b.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c5/b.log)"
  done
  timeout -k 10 300 python bench.py --config cfg3 --cpu-baseline-seconds 0 > gpurun_out/c5/b3.log 2>&1 || { tail -5 gpurun_out/c5/b3.log; exit 1; }
  echo "cfg3 $r $(grep -o '"value": [0-9.]*' gpurun_out/c5/b3.log | head -1)"
done
