set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_unrolled_gpu.py tests/test_sas_gpu.py tests/test_dp_gpu.py tests/test_sampler_gpu.py tests/test_itemgrad_gpu.py > gpurun_out/g17_tests.log 2>&1
for r in a b; do for E in 0 1; do RS_SAS_EMB_GRAD_SIDE=$E timeout -k 10 200 python bench.py --config cfg2 --cpu-baseline-seconds 0 > gpurun_out/g17_cfg2_e${E}$r.json 2>> gpurun_out/g17.err; done; done
timeout -k 10 200 python bench.py --config cfg4 --cpu-baseline-seconds 0 --steps-per-graph 1 > gpurun_out/g17_cfg4_s1.json 2>> gpurun_out/g17.err
timeout -k 10 200 python bench.py --config cfg4 --cpu-baseline-seconds 0 --steps-per-graph 4 > gpurun_out/g17_cfg4_s4.json 2>> gpurun_out/g17.err
