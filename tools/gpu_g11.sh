set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; OUT=gpurun_out/g11; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_wgrad_gpu.py tests/test_bert.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_w.log 2>&1; rc=$?; tail -2 $OUT/pytest_w.log; [ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-cfg3 cfg2}; do
  timeout -k 10 300 python bench.py --config $c --cpu-baseline-seconds 0 > $OUT/bench_$c.log 2>&1 || { tail -20 $OUT/bench_$c.log; exit 1; }
  tail -1 $OUT/bench_$c.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());r=d['roofline'];print('$c',d['value'],d['ms_per_step'],r['avg_launch_us'],r['isolated_launch_us'],r['frac'])"
done
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d $OUT/traffic_$P -o pmc --output-format csv -- python3 tools/kbench.py --config cfg3 --reps 5 --only "wgrad_grouped" > $OUT/traffic_$P.log 2>&1 || { tail -5 $OUT/traffic_$P.log; exit 1; }
done
mkdir -p $OUT/traffic && mv $OUT/traffic_FETCH_SIZE $OUT/traffic_WRITE_SIZE $OUT/traffic/ && python3 tools/make_traffic.py $OUT/traffic cfg3 $OUT/traffic.json && cat $OUT/traffic.json | head -5
echo done
