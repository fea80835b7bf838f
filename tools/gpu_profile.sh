#!/bin/bash
# rocprof kernel stats + one step's timeline per config, keeping only the small summaries (the raw trace
# directories are deleted: gpurun copies back at most 64 MiB).  CONFIGS="cfg2 cfg4" TAG=x bash tools/gpu_profile.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-prof}
mkdir -p $OUT
for c in ${CONFIGS:-cfg2}; do
  PS="--steps 50 --warmup 10"; [ "$c" = "cfg5" ] && PS="--steps 10 --warmup 3"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/raw_$c -o prof --output-format csv -- python3 bench.py --config $c $PS --cpu-baseline-seconds 0 $EXTRA > $OUT/rocprof_$c.log 2>&1 || { tail -20 $OUT/rocprof_$c.log; exit 1; }
  tail -1 $OUT/rocprof_$c.log | cut -c1-200
  cp "$(find $OUT/raw_$c -name '*kernel_stats.csv' | head -1)" $OUT/${c}_kernel_stats.csv
  python3 tools/step_timeline.py "$(find $OUT/raw_$c -name '*kernel_trace.csv' | head -1)" 3 > $OUT/${c}_step_timeline.txt || exit 1
  tail -1 $OUT/${c}_step_timeline.txt
  rm -rf $OUT/raw_$c
done
echo done
