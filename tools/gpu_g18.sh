set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_unrolled_gpu.py tests/test_sas_gpu.py tests/test_dp_gpu.py tests/test_sampler_gpu.py > gpurun_out/g18_tests.log 2>&1
for r in a b; do for E in 0 1; do RS_SAS_WGRAD_SIDE=$E timeout -k 10 200 python bench.py --config cfg2 --cpu-baseline-seconds 0 > gpurun_out/g18_cfg2_w${E}$r.json 2>> gpurun_out/g18.err; done; done
for E in 0 1; do RS_SAS_WGRAD_SIDE=$E timeout -k 10 200 python bench.py --config cfg3 --cpu-baseline-seconds 0 > gpurun_out/g18_cfg3_w${E}.json 2>> gpurun_out/g18.err; done
