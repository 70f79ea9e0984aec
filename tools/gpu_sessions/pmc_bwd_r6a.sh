# Round-4 PMC passes for the flash-attention backward kernels (S=8192, H=32, KV=8, D=128, causal):
# instruction mix and stall buckets per kernel, one counter pass per rocprofv3 run (--pmc only).
set -o pipefail
OUT=gpurun_out/pmc_r6a
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || echo "list rc=$?"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d $OUT -o p1 -- python3 tools/bench_attn.py > $OUT/p1.log 2>&1 || { echo "p1 rc=$?"; tail -5 $OUT/p1.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM --output-format csv -d $OUT -o p2 -- python3 tools/bench_attn.py > $OUT/p2.log 2>&1 || { echo "p2 rc=$?"; tail -5 $OUT/p2.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_TRANS_F32 SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_WAVES --output-format csv -d $OUT -o p3 -- python3 tools/bench_attn.py > $OUT/p3.log 2>&1 || { echo "p3 rc=$?"; tail -5 $OUT/p3.log; }
timeout -k 10 120 python3 tools/bench_attn.py > $OUT/bench_attn.log 2>&1
ls $OUT
