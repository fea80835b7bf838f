set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_unrolled_gpu.py tests/test_sas_gpu.py tests/test_dp_gpu.py tests/test_sampler_gpu.py tests/test_checkpoint_gpu.py > gpurun_out/g31.log 2>&1
for r in a b; do for E in 0 1; do RS_SAS_POS_MERGED=$E timeout -k 10 200 python bench.py --config cfg2 --cpu-baseline-seconds 0 > gpurun_out/g31_cfg2_p${E}$r.json 2>> gpurun_out/g31.err; done; done
for E in 0 1; do RS_SAS_POS_MERGED=$E timeout -k 10 200 python bench.py --config cfg4 --cpu-baseline-seconds 0 > gpurun_out/g31_cfg4_p${E}.json 2>> gpurun_out/g31.err; done
