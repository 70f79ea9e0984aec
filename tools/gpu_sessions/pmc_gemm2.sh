# memory-path counters for the weight-gradient GEMM (own run: --pmc only)
set -o pipefail
mkdir -p gpurun_out/pmcg2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmcg2/avail.txt 2>&1 || true
export SHAPES=o DSTACK_AMD_GEMM_TN=plain
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum --output-format csv -d gpurun_out/pmcg2 -o m1 -- python3 tools/bench_gemm.py > gpurun_out/pmcg2/run1.log 2>&1
echo "m1 rc=$?"
timeout -k 10 300 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum --output-format csv -d gpurun_out/pmcg2 -o m2 -- python3 tools/bench_gemm.py > gpurun_out/pmcg2/run2.log 2>&1
echo "m2 rc=$?"
ls gpurun_out/pmcg2
