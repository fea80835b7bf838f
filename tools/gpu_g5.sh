set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; OUT=gpurun_out/g5; mkdir -p $OUT
timeout -k 10 300 python tools/vhead_bench.py > $OUT/vb.log 2>&1; rc=$?; cat $OUT/vb.log; [ $rc -eq 0 ] || exit $rc
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d $OUT/pmc_$i -o pmc --output-format csv -- python3 tools/vhead_bench.py --reps 2 --only fwd,bwd > $OUT/pmc_$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/pmc_$i.log; exit 1; }
done
echo done
