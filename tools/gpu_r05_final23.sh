#!/bin/bash
# Round-5 closing pass for cfg2 / cfg3 at HEAD: bench lines (CPU baselines included), rocprof stats / step timelines,
# and the driver's own command shape for cfg2 (gpurun_out/r05e).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r05e
mkdir -p $OUT
for c in cfg2 cfg3; do
  timeout -k 10 600 python bench.py --config $c --cpu-baseline-seconds 10 > $OUT/bench_$c.log 2>&1 || { tail -5 $OUT/bench_$c.log; exit 1; }
  tail -1 $OUT/bench_$c.log > $OUT/bench_$c.json
  cut -c1-150 $OUT/bench_$c.json
done
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/drv_$r.log 2>&1 || exit 1
  echo "driver shape $r: $(grep -o '"value": [0-9.]*' $OUT/drv_$r.log | head -1)"
done
CONFIGS="cfg2 cfg3" TAG=r05e bash tools/gpu_profile.sh
