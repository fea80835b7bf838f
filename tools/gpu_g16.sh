set -e
mkdir -p gpurun_out
true
for S in 1 4 8; do timeout -k 10 200 python bench.py --config cfg2 --cpu-baseline-seconds 0 --steps-per-graph $S > gpurun_out/g16_cfg2_s$S.json 2> gpurun_out/g16_cfg2_s$S.err; done
timeout -k 10 200 python bench.py --config cfg2 --cpu-baseline-seconds 0 --steps-per-graph 1 > gpurun_out/g16_cfg2_s1b.json 2>> gpurun_out/g16_cfg2_s1.err
timeout -k 10 200 python bench.py --config cfg2 --cpu-baseline-seconds 0 --steps-per-graph 4 > gpurun_out/g16_cfg2_s4b.json 2>> gpurun_out/g16_cfg2_s4.err
timeout -k 10 200 python bench.py --config cfg4 --cpu-baseline-seconds 0 --steps-per-graph 1 > gpurun_out/g16_cfg4_s1.json 2> gpurun_out/g16_cfg4.err
timeout -k 10 200 python bench.py --config cfg4 --cpu-baseline-seconds 0 --steps-per-graph 4 > gpurun_out/g16_cfg4_s4.json 2>> gpurun_out/g16_cfg4.err
