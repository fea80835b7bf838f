set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_unrolled_gpu.py > gpurun_out/g32.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p32 -o prof --output-format csv -- python3 bench.py --config cfg2 --steps 40 --warmup 8 --cpu-baseline-seconds 0 > gpurun_out/p32.log 2>&1
for r in a b; do timeout -k 10 200 python bench.py --config cfg2 --cpu-baseline-seconds 0 > gpurun_out/g32_cfg2_$r.json; done
