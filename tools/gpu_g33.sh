set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_unrolled_gpu.py tests/test_bench_gpu.py tests/test_sampler_gpu.py > gpurun_out/g33.log 2>&1
for r in a b c; do timeout -k 10 200 python bench.py --config cfg2 --cpu-baseline-seconds 0 > gpurun_out/g33_cfg2_$r.json; done
timeout -k 10 200 python bench.py --config cfg4 --cpu-baseline-seconds 0 > gpurun_out/g33_cfg4.json
