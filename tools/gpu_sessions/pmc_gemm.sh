# PMC counters for the weight-gradient GEMM kernel (own run: --pmc only, no tracing domains)
set -o pipefail
mkdir -p gpurun_out/pmcg
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export SHAPES=o DSTACK_AMD_GEMM_TN=${DSTACK_AMD_GEMM_TN:-plain}
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmcg -o g1 -- python3 tools/bench_gemm.py > gpurun_out/pmcg/run1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_VMEM GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcg -o g2 -- python3 tools/bench_gemm.py > gpurun_out/pmcg/run2.log 2>&1
echo "pmc rc=$?"
ls gpurun_out/pmcg
