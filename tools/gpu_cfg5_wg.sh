#!/bin/bash
# cfg5: workgroup cap of the token table's early optimizer update (RS_EARLY_TOKEN_ADAM_WG), interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c5wg
for r in 1 2; do
  for w in 256 512 1024 2048; do
    RS_EARLY_TOKEN_ADAM_WG=$w timeout -k 10 300 python bench.py --config cfg5 --steps 30 --warmup 5 --cpu-baseline-seconds 0 > gpurun_out/c5wg/b.log 2>&1 || { tail -5 gpurun_out/c5wg/b.log; exit 1; }
    echo "cfg5 $r wg=$w $(grep -o '"value": [0-9.]*' gpurun_out/c5wg/b.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c5wg/b.log)"
  done
done
