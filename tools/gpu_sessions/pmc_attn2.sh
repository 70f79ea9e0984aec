# PMC counters for the flash-attention kernels at S=8192 (own runs: --pmc only, no tracing domains)
set -o pipefail
mkdir -p gpurun_out/pmc2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc2 -o sq -- python3 tools/bench_attn.py > gpurun_out/pmc2/sq.log 2>&1 || { echo "sq pass rc=$?"; tail -5 gpurun_out/pmc2/sq.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --output-format csv -d gpurun_out/pmc2 -o tcc -- python3 tools/bench_attn.py > gpurun_out/pmc2/tcc.log 2>&1 || { echo "tcc pass rc=$?"; tail -5 gpurun_out/pmc2/tcc.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv -d gpurun_out/pmc2 -o tcc2 -- python3 tools/bench_attn.py > gpurun_out/pmc2/tcc2.log 2>&1 || { echo "tcc2 pass rc=$?"; tail -5 gpurun_out/pmc2/tcc2.log; exit 1; }
ls gpurun_out/pmc2
