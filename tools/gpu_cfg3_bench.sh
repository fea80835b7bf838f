#!/bin/bash
# cfg3 bench line (with its CPU baseline), reading the round's PMC traffic from profiles/traffic.json.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r05c
timeout -k 10 900 python bench.py --config cfg3 --cpu-baseline-seconds 10 > gpurun_out/r05c/bench_cfg3.log 2>&1 || { tail -5 gpurun_out/r05c/bench_cfg3.log; exit 1; }
tail -1 gpurun_out/r05c/bench_cfg3.log > gpurun_out/r05c/bench_cfg3.json
