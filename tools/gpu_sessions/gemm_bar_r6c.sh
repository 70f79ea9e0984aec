# The forward GEMMs' speed at the step shapes (the bar for an owned fused-epilogue GEMM), then
# one PMC pass over the same program for MFMA busy / wave cycles
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/gemm_bar_r6c
cd $R
for i in 1 2 3; do
  timeout -k 10 200 python tools/bench_fwd_gemms.py > gpurun_out/gemm_bar_r6c/run_$i.json 2>gpurun_out/gemm_bar_r6c/err.log || exit 1
  cat gpurun_out/gemm_bar_r6c/run_$i.json
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/gemm_bar_r6c/pmc -o p -- python3 $R/tools/bench_fwd_gemms.py > $R/gpurun_out/gemm_bar_r6c/pmc.log 2>&1 || exit 1
echo pmc done
