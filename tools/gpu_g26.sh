set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_itemgrad_gpu.py tests/test_wgrad_gpu.py tests/test_sas_gpu.py tests/test_unrolled_gpu.py tests/test_dp_gpu.py tests/test_adam_gpu.py tests/test_sampler_gpu.py > gpurun_out/g26.log 2>&1
for r in a b; do for E in side fused; do RS_SAS_GRAD_TAIL=$E timeout -k 10 200 python bench.py --config cfg2 --cpu-baseline-seconds 0 > gpurun_out/g26_cfg2_${E}$r.json 2>> gpurun_out/g26.err; done; done
for E in side fused; do RS_SAS_GRAD_TAIL=$E timeout -k 10 200 python bench.py --config cfg4 --cpu-baseline-seconds 0 > gpurun_out/g26_cfg4_${E}.json 2>> gpurun_out/g26.err; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p26 -o prof --output-format csv -- python3 bench.py --config cfg2 --steps 40 --warmup 8 --cpu-baseline-seconds 0 > gpurun_out/p26.log 2>&1
