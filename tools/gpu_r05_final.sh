#!/bin/bash
# Round-5 closing pass: the GPU suite + smoke, then the cfg4 / cfg5 bench lines (CPU baselines included) and their
# rocprof stats / step timelines (gpurun_out/r05d).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r05d
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -2 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "__import__('__graft_entry__').smoke()" > $OUT/smoke.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/smoke.log
timeout -k 10 600 python bench.py --config cfg4 --cpu-baseline-seconds 10 > $OUT/bench_cfg4.log 2>&1 || { tail -5 $OUT/bench_cfg4.log; exit 1; }
tail -1 $OUT/bench_cfg4.log > $OUT/bench_cfg4.json
timeout -k 10 900 python bench.py --config cfg5 --cpu-baseline-seconds 10 --steps 30 --warmup 5 > $OUT/bench_cfg5.log 2>&1 || { tail -5 $OUT/bench_cfg5.log; exit 1; }
tail -1 $OUT/bench_cfg5.log > $OUT/bench_cfg5.json
cut -c1-160 $OUT/bench_cfg4.json $OUT/bench_cfg5.json
CONFIGS="cfg4 cfg5" TAG=r05d bash tools/gpu_profile.sh
