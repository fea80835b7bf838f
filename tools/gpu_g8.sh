set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; OUT=gpurun_out/g8; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_dp_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_dp.log 2>&1; rc=$?; tail -16 $OUT/pytest_dp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
echo done
