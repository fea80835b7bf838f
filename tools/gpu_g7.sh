set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; OUT=gpurun_out/g7; mkdir -p $OUT
for D in 0 1 2 4 7; do
  echo "dbg $D"; RS_VHEAD_DBG=$D timeout -k 10 120 python tools/vhead_bench.py --only fwd,bwd 2>&1 | grep vocab
done
echo "R=128"; timeout -k 10 120 python tools/vhead_bench.py --only fwd,bwd --R 128 2>&1 | grep vocab
echo "R=512"; timeout -k 10 120 python tools/vhead_bench.py --only fwd,bwd --R 512 2>&1 | grep vocab
echo done
