#!/bin/bash
# Phase stamps of the row-chain block_out and the attention backward (tools/micro, built on the CPU side),
# then the cfg2 bench in the driver's shape and the long default.  TAG=x bash tools/gpu_phase.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-phase}
mkdir -p $OUT
timeout -k 10 60 ./tools/micro/rowchain_phase 25600 > $OUT/rowchain_phase.txt 2>&1 || { cat $OUT/rowchain_phase.txt; exit 1; }
cat $OUT/rowchain_phase.txt
timeout -k 10 60 ./tools/micro/attn_bwd_phase > $OUT/attn_bwd_phase.txt 2>&1 || { cat $OUT/attn_bwd_phase.txt; exit 1; }
cat $OUT/attn_bwd_phase.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 > $OUT/bench20.log 2>&1 || { tail -20 $OUT/bench20.log; exit 1; }
tail -1 $OUT/bench20.log | cut -c1-400
timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-400
