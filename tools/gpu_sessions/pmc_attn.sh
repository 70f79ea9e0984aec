# PMC counters for the flash-attention kernels (own run: --pmc only, no tracing domains)
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export S=4096
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc -o attn -- python3 tools/bench_attn.py > gpurun_out/pmc/run.log 2>&1
echo "pmc rc=$?"
ls gpurun_out/pmc
