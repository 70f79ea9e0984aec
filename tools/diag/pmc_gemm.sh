#!/bin/bash
# PMC passes over tools/bench_gemm_nt.py for a few shapes (our gemm_nt vs hipBLASLt), one pass per run.
# usage: bash tools/diag/pmc_gemm.sh <outdir> [SHAPES]
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=${1:-gpurun_out/pmc_gemm}
export SHAPES=${2:-fwd_o,dgrad_lm} ROUNDS=1 ITERS=3
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 tools/bench_gemm_nt.py > $OUT/trace.log 2>&1
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P -d $OUT/p$i -o run -- python3 tools/bench_gemm_nt.py > $OUT/p$i.log 2>&1
done
python3 tools/pmc_summary.py $(find $OUT -name "*counter_collection.csv") > $OUT/summary.txt
cat $OUT/summary.txt
find $OUT/trace -name "*kernel_stats.csv" -exec cat {} \; | head -20
