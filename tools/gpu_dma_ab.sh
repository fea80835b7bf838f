#!/bin/bash
# DMA GEMM / grouped weight-gradient check on the GPU box: bitwise tests, the cfg3-shape GEMM A/B (register-staged vs
# DMA 128 / 64-row tiles), the grouped weight gradients (kbench) and whole steps with each form.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-dma}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_dma_gpu.py tests/test_wgrad_gpu.py tests/test_bert.py -k 'dma or wgrad or early_head' > $OUT/test.log 2>&1; rc=$?; tail -3 $OUT/test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/diag/gemm_epi.py --reps 50 --envs 'RS_GEMM_DMA=0;RS_GEMM_DMA=1,RS_GEMM_DMA_BM=128;RS_GEMM_DMA=1,RS_GEMM_DMA_BM=64' > $OUT/gemm_epi.log 2>&1 || exit $?
for c in cfg2 cfg3; do for f in 0 1; do
  ONLY=wgrad_grouped
  RS_WGRAD_DMA=$f timeout -k 10 200 python tools/kbench.py --config $c --reps 50 --only "$ONLY" > $OUT/kb_${c}_$f.log 2>&1 || exit $?
done; done
for c in cfg3 cfg2; do
  RS_GEMM_DMA=0 RS_WGRAD_DMA=0 timeout -k 10 300 python bench.py --config $c --cpu-baseline-seconds 0 > $OUT/bench_${c}_old.log 2>&1 || exit $?
  RS_GEMM_DMA=1 RS_WGRAD_DMA=1 timeout -k 10 300 python bench.py --config $c --cpu-baseline-seconds 0 > $OUT/bench_${c}_new.log 2>&1 || exit $?
  RS_GEMM_DMA=0 RS_WGRAD_DMA=0 timeout -k 10 300 python bench.py --config $c --cpu-baseline-seconds 0 > $OUT/bench_${c}_old2.log 2>&1 || exit $?
  RS_GEMM_DMA=1 RS_WGRAD_DMA=1 timeout -k 10 300 python bench.py --config $c --cpu-baseline-seconds 0 > $OUT/bench_${c}_new2.log 2>&1 || exit $?
done
for f in 0 1; do
  RS_EARLY_HEAD_ADAM=$f RS_GEMM_DMA=1 RS_WGRAD_DMA=1 timeout -k 10 400 python bench.py --config cfg5 --steps 30 --warmup 5 --cpu-baseline-seconds 0 > $OUT/bench_cfg5_early$f.log 2>&1 || exit $?
done
grep -h "" $OUT/gemm_epi.log | tail -60
for f in $OUT/kb_*.log; do echo "== $f"; tail -4 $f; done
for f in $OUT/bench_*.log; do echo "== $f"; tail -1 $f | cut -c1-120; done
