set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for B in 8192 256 512; do RS_ADAM_PREP_BLOCKS=$B timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p22_$B -o prof --output-format csv -- python3 bench.py --config cfg2 --steps 40 --warmup 8 --cpu-baseline-seconds 0 > gpurun_out/p22_$B.log 2>&1; done
