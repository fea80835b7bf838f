set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; OUT=gpurun_out/g6; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_bert.py -m gpu -x -q --timeout 120 --timeout-method thread -k vocab > $OUT/pytest_vocab.log 2>&1; rc=$?; tail -3 $OUT/pytest_vocab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/vhead_bench.py $VB_ARGS > $OUT/vb.log 2>&1; rc=$?; cat $OUT/vb.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
if [ -n "$PMC" ]; then
P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P2 -d $OUT/pmc_2 -o pmc --output-format csv -- python3 tools/vhead_bench.py --reps 2 --only fwd,bwd > $OUT/pmc_2.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/pmc_2.log; exit 1; }
fi
echo done
