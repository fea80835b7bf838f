set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; OUT=gpurun_out/g9; mkdir -p $OUT
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --cpu-baseline-seconds 0 > $OUT/dp2.log 2>&1 || { tail -30 $OUT/dp2.log; exit 1; }
tail -1 $OUT/dp2.log | cut -c1-400
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --config cfg3 --steps 10 --warmup 3 --dist-backend gloo --cpu-baseline-seconds 0 > $OUT/dp2b.log 2>&1 || { tail -30 $OUT/dp2b.log; exit 1; }
tail -1 $OUT/dp2b.log | cut -c1-400
echo done
