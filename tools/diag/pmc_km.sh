#!/bin/bash
# KM vs NT form of the in-tree GEMM on one weight-gradient shape: timings (store / no-store) and
# three --pmc passes (one per run) over tools/diag/km_vs_nt.py.
# usage: bash tools/diag/pmc_km.sh <outdir> [M,N,K]
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=${1:-gpurun_out/pmc_km}
export SHAPE=${2:-28672,4096,8192} ROUNDS=3
mkdir -p $OUT
timeout -k 10 120 python3 -u tools/diag/km_vs_nt.py > $OUT/timing.log 2>&1
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 tools/diag/km_vs_nt.py > $OUT/p$i.log 2>&1
done
python3 tools/pmc_summary.py $(find $OUT -name "*counter_collection.csv") > $OUT/summary.txt
cat $OUT/timing.log $OUT/summary.txt
