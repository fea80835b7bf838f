set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; OUT=gpurun_out/g1; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 > $OUT/bench2.log 2>&1 || { tail -20 $OUT/bench2.log; exit 1; }
tail -1 $OUT/bench2.log
timeout -k 10 300 python bench.py --config cfg4 --cpu-baseline-seconds 0 > $OUT/bench4.log 2>&1 || { tail -20 $OUT/bench4.log; exit 1; }
tail -1 $OUT/bench4.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof2 -o prof --output-format csv -- python3 bench.py --steps 50 --warmup 10 --cpu-baseline-seconds 0 > $OUT/rocprof2.log 2>&1 || { tail -20 $OUT/rocprof2.log; exit 1; }
echo done
