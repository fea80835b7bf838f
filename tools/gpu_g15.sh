set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; OUT=gpurun_out/g15; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --config cfg5 --steps 5 --warmup 2 --dist-backend gloo --cpu-baseline-seconds 0 > $OUT/dp5.log 2>&1 || { tail -30 $OUT/dp5.log; exit 1; }
tail -1 $OUT/dp5.log | cut -c1-300; tail -1 $OUT/dp5.log | grep -o '"vocab_sharded_head": true'
echo done
