set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; OUT=gpurun_out/g4; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_bert.py -m gpu -x -q --timeout 120 --timeout-method thread -k vocab > $OUT/pytest_vocab.log 2>&1; rc=$?; tail -15 $OUT/pytest_vocab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-cfg3 cfg5}; do
  ST=200; [ $c = cfg5 ] && ST=20
  timeout -k 10 600 python bench.py --config $c --steps $ST --cpu-baseline-seconds 0 > $OUT/bench_$c.log 2>&1 || { tail -20 $OUT/bench_$c.log; exit 1; }
  tail -1 $OUT/bench_$c.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());r=d['roofline'];print('$c',d['value'],d['ms_per_step'],d['final_loss'],r['kernel'][:30],r['avg_launch_us'],r['isolated_launch_us'],r['frac'])"
done
if [ -n "$PROF" ]; then
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$PROF -o prof --output-format csv -- python3 bench.py --config $PROF --steps 10 --warmup 3 --cpu-baseline-seconds 0 > $OUT/rocprof.log 2>&1 || { tail -20 $OUT/rocprof.log; exit 1; }
fi
echo done
