set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_itemgrad_gpu.py tests/test_sas_gpu.py tests/test_unrolled_gpu.py tests/test_sampler_gpu.py > gpurun_out/g29.log 2>&1
for r in a b c; do timeout -k 10 200 python bench.py --config cfg2 --cpu-baseline-seconds 0 > gpurun_out/g29_cfg2_$r.json 2>> gpurun_out/g29.err; done
timeout -k 10 200 python bench.py --config cfg4 --cpu-baseline-seconds 0 > gpurun_out/g29_cfg4.json 2>> gpurun_out/g29.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p29 -o prof --output-format csv -- python3 bench.py --config cfg2 --steps 40 --warmup 8 --cpu-baseline-seconds 0 > gpurun_out/p29.log 2>&1
