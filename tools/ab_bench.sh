#!/bin/bash
# A/B timing in one GPU session, alternating, CONFIG (default cfg2), ROUNDS (default 3):
#   A = librecsys_hip.$A.so (RS_LIB_VARIANT=$A), or with AENV="NAME=value" the in-tree library under that setting;
#   B = the in-tree librecsys_hip.so as is.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for i in $(seq ${ROUNDS:-3}); do
  for v in A B; do
    if [ $v = A ] && [ -n "$AENV" ]; then envs="$AENV"; elif [ $v = A ]; then envs="RS_LIB_VARIANT=${A:-a}"; else envs="RS_AB_B=1"; fi
    env $envs timeout -k 10 200 python bench.py --config ${CONFIG:-cfg2} --steps 200 --warmup 20 \
      --cpu-baseline-seconds 0 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.log) $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/ab.log)"
  done
done
