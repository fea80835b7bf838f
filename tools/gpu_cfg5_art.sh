#!/bin/bash
# cfg5 round artifacts only: the bench line (with its CPU baseline) and the rocprof stats / step timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05b}
mkdir -p $OUT
timeout -k 10 900 python bench.py --config cfg5 --cpu-baseline-seconds ${CPU_SECONDS_OTHER:-10} --steps 30 --warmup 5 > $OUT/bench_cfg5.log 2>&1 || { tail -5 $OUT/bench_cfg5.log; exit 1; }
tail -1 $OUT/bench_cfg5.log > $OUT/bench_cfg5.json
cut -c1-200 $OUT/bench_cfg5.json
CONFIGS=cfg5 TAG=${TAG:-r05b} bash tools/gpu_profile.sh || exit 1
