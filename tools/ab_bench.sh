#!/bin/bash
# A/B timing of two library builds in one GPU session: librecsys_hip.$A.so (RS_LIB_VARIANT=$A) against the
# in-tree librecsys_hip.so, alternating, CONFIG (default cfg2), ROUNDS (default 3).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for i in $(seq ${ROUNDS:-3}); do
  for v in "${A:-a}" ""; do
    RS_LIB_VARIANT=$v timeout -k 10 200 python bench.py --config ${CONFIG:-cfg2} --steps 200 --warmup 20 \
      --cpu-baseline-seconds 0 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    echo "${v:-B} $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.log) $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/ab.log)"
  done
done
