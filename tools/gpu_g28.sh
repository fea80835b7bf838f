set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in a b; do for E in normal high; do RS_SAS_SIDE_PRIORITY=$E timeout -k 10 200 python bench.py --config cfg2 --cpu-baseline-seconds 0 > gpurun_out/g28_cfg2_${E}$r.json 2>> gpurun_out/g28.err; done; done
RS_SAS_SIDE_PRIORITY=high timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p28 -o prof --output-format csv -- python3 bench.py --config cfg2 --steps 40 --warmup 8 --cpu-baseline-seconds 0 > gpurun_out/p28.log 2>&1
