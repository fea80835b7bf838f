#!/bin/bash
# PMC counter passes (one rocprofv3 run per pass, --kernel-trace only beside --pmc) over
# tools/kbench.py --only "$ONLY" (default: fused kernels).  Output: gpurun_out/$TAG/pmc_<pass>/...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc}
mkdir -p $OUT
ONLY=${ONLY:-fused}
CFG=${CFG:-cfg2}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM"
P3="FETCH_SIZE"
P4="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P -d $OUT/pmc_$i -o pmc --output-format csv -- python3 tools/kbench.py --config $CFG --reps 5 --only "$ONLY" > $OUT/pmc_$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/pmc_$i.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
