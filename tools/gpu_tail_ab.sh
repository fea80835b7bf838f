#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tail
for i in 1 2; do
  for m in side main_before main_after; do
    RS_SAS_TAIL=$m timeout -k 10 200 python bench.py --config cfg2 --steps 200 --warmup 20 --cpu-baseline-seconds 0 > gpurun_out/tail/ab.log 2>&1 || { tail -5 gpurun_out/tail/ab.log; exit 1; }
    echo "$m $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tail/ab.log)"
  done
done
for m in main_before main_after; do
  RS_SAS_TAIL=$m CONFIGS=cfg2 TAG=tail/$m bash tools/gpu_profile.sh > /dev/null 2>&1 || exit 1
  tail -9 gpurun_out/tail/$m/cfg2_step_timeline.txt
done
