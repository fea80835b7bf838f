#!/bin/bash
# Round artifacts on the GPU box: GPU tests, HBM traffic of the roofline kernel (PMC passes ->
# traffic.json), the default bench line per config (with the CPU baseline), rocprof kernel stats.
# Everything lands under gpurun_out/$TAG; copy what is judged into profiles/ afterwards.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-art}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
rm -f profiles/traffic.json
for c in cfg2 cfg3 cfg4; do
  ONLY=attn_bwd; [ "$c" = "cfg3" ] && ONLY="bert wgrad_grouped"
  for P in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P -d $OUT/traffic_${c}_$P -o pmc --output-format csv -- python3 tools/kbench.py --config $c --reps 5 --only "$ONLY" > $OUT/traffic_${c}_$P.log 2>&1 || { tail -5 $OUT/traffic_${c}_$P.log; exit 1; }
  done
  mkdir -p $OUT/traffic_$c && mv $OUT/traffic_${c}_FETCH_SIZE $OUT/traffic_${c}_WRITE_SIZE $OUT/traffic_$c/
  python3 tools/make_traffic.py $OUT/traffic_$c $c profiles/traffic.json > /dev/null || exit 1
done
cp profiles/traffic.json $OUT/traffic.json
for c in ${CONFIGS:-cfg2 cfg3 cfg4 cfg5}; do
  CB=""; [ "$c" != "cfg2" ] && CB="--cpu-baseline-seconds ${CPU_SECONDS_OTHER:-10}"
  ST=""; [ "$c" = "cfg5" ] && ST="--steps 30 --warmup 5"
  timeout -k 10 900 python bench.py --config $c $CB $ST > $OUT/bench_$c.log 2>&1; rc=$?; tail -1 $OUT/bench_$c.log | cut -c1-160
  [ $rc -eq 0 ] || exit $rc
  tail -1 $OUT/bench_$c.log > $OUT/bench_$c.json
done
# rocprof kernel stats + one step's timeline per config (raw traces deleted: gpurun copies back <= 64 MiB)
CONFIGS="${CONFIGS:-cfg2 cfg3 cfg4 cfg5}" TAG=${TAG:-art} bash tools/gpu_profile.sh || exit 1
echo done
