#!/bin/bash
# The one GPU-box script: every committed profile under profiles/ names the mode of this script that made it.
# Output lands under gpurun_out/$TAG (scratch); copy what is judged into profiles/ afterwards.  Every GPU step runs
# under its own time limit and the chain stops at the first failure (after a timeout / abort / fault nothing more
# runs on the GPU in that call).
#
#   bash tools/gpu.sh suite                      pytest -m gpu, then __graft_entry__.smoke()
#   bash tools/gpu.sh tests <pytest args...>     a subset of the GPU tests
#   bash tools/gpu.sh bench cfg2 cfg4 ...        the default bench line per config (CPU baseline included)
#   bash tools/gpu.sh profile cfg2 ...           rocprofv3 --kernel-trace --stats of bench.py + one step's timeline
#   bash tools/gpu.sh traffic cfg2 cfg3 cfg4     HBM bytes of the roofline kernels (FETCH_SIZE / WRITE_SIZE passes)
#                                                -> profiles/traffic.json
#   bash tools/gpu.sh pmc CFG "ONLY"             the four PMC counter passes over tools/kbench.py --only ONLY
#   bash tools/gpu.sh ab CFG                     interleaved A/B: A = librecsys_hip.$A.so (RS_LIB_VARIANT, see
#                                                tools/build_variant.sh) or the in-tree library under AENV="X=1";
#                                                B = the in-tree library.  ROUNDS (3), STEPS (200)
#   bash tools/gpu.sh artifacts                  suite, traffic, bench and profile of cfg2..cfg5 (round close)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-gpu}
mkdir -p "$OUT"
mode=$1
shift

suite() {
  timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; return 1; }
  tail -2 "$OUT/pytest_gpu.log"
  timeout -k 10 300 python -c "__import__('__graft_entry__').smoke()" > "$OUT/smoke.log" 2>&1 \
    || { tail -20 "$OUT/smoke.log"; return 1; }
  grep -v amdgpu.ids "$OUT/smoke.log"
}

tests() {
  timeout -k 10 ${LIMIT:-900} python -u -m pytest -x -v -rP --timeout 240 --timeout-method thread "$@" \
    > "$OUT/pytest.log" 2>&1; rc=$?
  grep -E "PASSED|FAILED|ERROR|passed|failed" "$OUT/pytest.log" | tail -${TAILN:-40}
  return $rc
}

bench() {
  for c in "$@"; do
    local st=""; [ "$c" = "cfg5" ] && st="--steps 30 --warmup 5"
    timeout -k 10 900 python bench.py --config "$c" $st ${BENCH_ARGS:-} > "$OUT/bench_$c.log" 2>&1 \
      || { tail -20 "$OUT/bench_$c.log"; return 1; }
    tail -1 "$OUT/bench_$c.log" > "$OUT/bench_$c.json"
    cut -c1-200 "$OUT/bench_$c.json"
  done
}

profile() {
  for c in "$@"; do
    local ps="--steps 50 --warmup 10"; [ "$c" = "cfg5" ] && ps="--steps 10 --warmup 3"
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/raw_$c" -o prof --output-format csv -- \
      python3 bench.py --config "$c" $ps --cpu-baseline-seconds 0 ${BENCH_ARGS:-} > "$OUT/rocprof_$c.log" 2>&1 \
      || { tail -20 "$OUT/rocprof_$c.log"; return 1; }
    tail -1 "$OUT/rocprof_$c.log" > "$OUT/prof_bench_$c.json"
    cp "$(find "$OUT/raw_$c" -name '*kernel_stats.csv' | head -1)" "$OUT/${c}_kernel_stats.csv"
    python3 tools/step_timeline.py "$(find "$OUT/raw_$c" -name '*kernel_trace.csv' | head -1)" 3 \
      > "$OUT/${c}_step_timeline.txt" || return 1
    tail -1 "$OUT/${c}_step_timeline.txt"
    rm -rf "$OUT/raw_$c"           # gpurun copies back at most 64 MiB
  done
}

traffic() {
  for c in "$@"; do
    local only=attn_bwd; [ "$c" = "cfg3" ] && only="bert wgrad_grouped"
    for p in FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 300 rocprofv3 --kernel-trace --pmc $p -d "$OUT/traffic_${c}/$p" -o pmc --output-format csv -- \
        python3 tools/kbench.py --config "$c" --reps 5 --only "$only" > "$OUT/traffic_${c}_$p.log" 2>&1 \
        || { tail -5 "$OUT/traffic_${c}_$p.log"; return 1; }
    done
    python3 tools/make_traffic.py "$OUT/traffic_$c" "$c" profiles/traffic.json > /dev/null || return 1
  done
  cp profiles/traffic.json "$OUT/traffic.json"
}

pmc() {
  local cfg=$1 only=${2:-fused} i=0
  local p1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
  local p2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM"
  for p in "$p1" "$p2" "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $p -d "$OUT/pmc_$i" -o pmc --output-format csv -- \
      python3 tools/kbench.py --config "$cfg" --reps 5 --only "$only" > "$OUT/pmc_$i.log" 2>&1 \
      || { echo "pass $i failed"; tail -5 "$OUT/pmc_$i.log"; return 1; }
  done
  python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt"
}

ab() {
  local cfg=${1:-cfg2} envs
  for i in $(seq ${ROUNDS:-3}); do
    for v in A B; do
      if [ $v = A ] && [ -n "$AENV" ]; then envs="$AENV"; elif [ $v = A ]; then envs="RS_LIB_VARIANT=${A:-a}"
      else envs="RS_AB_B=1"; fi
      env $envs timeout -k 10 300 python bench.py --config "$cfg" --steps ${STEPS:-200} --warmup 20 \
        --cpu-baseline-seconds 0 ${BENCH_ARGS:-} > "$OUT/ab.log" 2>&1 || { tail -5 "$OUT/ab.log"; return 1; }
      echo "$v $(grep -o '"ms_per_step": [0-9.]*' "$OUT/ab.log") $(grep -o '"avg_launch_us": [0-9.]*' "$OUT/ab.log")"
    done
  done
}

case "$mode" in
  suite) suite ;;
  tests) tests "$@" ;;
  bench) bench "$@" ;;
  profile) profile "$@" ;;
  traffic) traffic "$@" ;;
  pmc) pmc "$@" ;;
  ab) ab "$@" ;;
  artifacts) suite && traffic cfg2 cfg3 cfg4 && bench cfg2 cfg3 cfg4 cfg5 && profile cfg2 cfg3 cfg4 cfg5 ;;
  *) sed -n 2,20p "$0"; exit 2 ;;
esac
