set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_adam_gpu.py tests/test_sas_gpu.py tests/test_dp_gpu.py tests/test_unrolled_gpu.py tests/test_checkpoint_gpu.py tests/test_trainer_dropin_gpu.py tests/test_sampler_gpu.py tests/test_curves_gpu.py > gpurun_out/g24.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p24 -o prof --output-format csv -- python3 bench.py --config cfg2 --steps 40 --warmup 8 --cpu-baseline-seconds 0 > gpurun_out/p24.log 2>&1
timeout -k 10 200 python bench.py --config cfg2 --cpu-baseline-seconds 0 > gpurun_out/g24_cfg2a.json
timeout -k 10 200 python bench.py --config cfg2 --cpu-baseline-seconds 0 > gpurun_out/g24_cfg2b.json
