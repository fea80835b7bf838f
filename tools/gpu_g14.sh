set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; OUT=gpurun_out/g14; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_vocab_shard_gpu.py -x -v --timeout 240 --timeout-method thread > $OUT/pytest_vs.log 2>&1; rc=$?; tail -30 $OUT/pytest_vs.log; [ $rc -eq 0 ] || exit $rc
echo done
