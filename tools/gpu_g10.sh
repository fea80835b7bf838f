set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; OUT=gpurun_out/g10; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py tests/test_sas_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_attn.log 2>&1; rc=$?; tail -3 $OUT/pytest_attn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/micro/attn_bwd_phase > $OUT/phase.log 2>&1; rc=$?; cat $OUT/phase.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for c in cfg2 cfg4; do
  timeout -k 10 300 python bench.py --config $c --cpu-baseline-seconds 0 > $OUT/bench_$c.log 2>&1 || { tail -20 $OUT/bench_$c.log; exit 1; }
  tail -1 $OUT/bench_$c.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());r=d['roofline'];print('$c',d['value'],d['ms_per_step'],r['avg_launch_us'],r['isolated_launch_us'],r['frac'])"
done
echo done
