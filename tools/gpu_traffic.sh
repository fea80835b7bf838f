# HBM traffic of the roofline kernels only (PMC passes -> profiles/traffic.json), as in gpu_artifacts.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-traffic}
mkdir -p $OUT
rm -f profiles/traffic.json
for c in cfg2 cfg3 cfg4; do
  ONLY=attn_bwd; [ "$c" = "cfg3" ] && ONLY="bert wgrad_grouped"
  for P in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P -d $OUT/traffic_${c}_$P -o pmc --output-format csv -- python3 tools/kbench.py --config $c --reps 5 --only "$ONLY" > $OUT/traffic_${c}_$P.log 2>&1 || { tail -5 $OUT/traffic_${c}_$P.log; exit 1; }
  done
  mkdir -p $OUT/traffic_$c && mv $OUT/traffic_${c}_FETCH_SIZE $OUT/traffic_${c}_WRITE_SIZE $OUT/traffic_$c/
  python3 tools/make_traffic.py $OUT/traffic_$c $c profiles/traffic.json > /dev/null || exit 1
done
cp profiles/traffic.json $OUT/traffic.json
for c in cfg2 cfg4; do timeout -k 10 300 python bench.py --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit 1; done
echo done
