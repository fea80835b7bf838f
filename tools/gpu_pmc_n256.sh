#!/bin/bash
# PMC passes over the cfg5-shape gemm_n256 launches (tools/diag/vocab_gemm_probe.py --only n256): one rocprofv3 run
# per counter pass.  Output gpurun_out/$TAG/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc256}
mkdir -p $OUT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM"
P3="FETCH_SIZE"
P4="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d $OUT/pmc_$i -o pmc --output-format csv -- python3 tools/diag/vocab_gemm_probe.py --only n256 --reps 3 > $OUT/pmc_$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/pmc_$i.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1; grep -A16 "gemm_n256" $OUT/summary.txt
