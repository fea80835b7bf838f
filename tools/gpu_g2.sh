set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; OUT=gpurun_out/g2; mkdir -p $OUT
timeout -k 10 300 python bench.py --sampler device --cpu-baseline-seconds 0 > $OUT/bench2dev.log 2>&1 || { tail -20 $OUT/bench2dev.log; exit 1; }
tail -1 $OUT/bench2dev.log | cut -c1-250
timeout -k 10 600 python bench.py --config cfg5 --steps 20 --warmup 5 --cpu-baseline-seconds 0 > $OUT/bench5.log 2>&1 || { tail -20 $OUT/bench5.log; exit 1; }
tail -1 $OUT/bench5.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof5 -o prof --output-format csv -- python3 bench.py --config cfg5 --steps 10 --warmup 3 --cpu-baseline-seconds 0 > $OUT/rocprof5.log 2>&1 || { tail -20 $OUT/rocprof5.log; exit 1; }
echo done
