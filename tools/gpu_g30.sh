set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_adam_gpu.py tests/test_checkpoint_gpu.py > gpurun_out/g30.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p30 -o prof --output-format csv -- python3 bench.py --config cfg5 --steps 10 --warmup 3 --cpu-baseline-seconds 0 > gpurun_out/p30.log 2>&1
timeout -k 10 300 python bench.py --config cfg5 --steps 30 --warmup 5 --cpu-baseline-seconds 0 > gpurun_out/g30_cfg5.json
for r in a b; do timeout -k 10 200 python bench.py --config cfg2 --cpu-baseline-seconds 0 > gpurun_out/g30_cfg2_$r.json; done
