set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py tests/test_sas_gpu.py tests/test_bert.py tests/test_unrolled_gpu.py > gpurun_out/g27.log 2>&1
for r in a b c; do timeout -k 10 200 python bench.py --config cfg2 --cpu-baseline-seconds 0 > gpurun_out/g27_cfg2_$r.json 2>> gpurun_out/g27.err; done
timeout -k 10 200 python bench.py --config cfg4 --cpu-baseline-seconds 0 > gpurun_out/g27_cfg4.json 2>> gpurun_out/g27.err
timeout -k 10 200 python bench.py --config cfg3 --cpu-baseline-seconds 0 > gpurun_out/g27_cfg3.json 2>> gpurun_out/g27.err
