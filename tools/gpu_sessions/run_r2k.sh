# cached W^T for the input-gradient GEMMs (TN layout): GPU op tests, tune the new shapes,
# same-box A/B, kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r2k.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_r2k.log | head -20; exit 1; }
tail -1 gpurun_out/gpu_tests_r2k.log
cp dstack_amd/ops/tuned/gemm_tunableop_gfx950.csv gpurun_out/tune_r2k.csv
DSTACK_AMD_GEMM_TUNING=tune DSTACK_AMD_GEMM_TUNING_FILE=gpurun_out/tune_r2k.csv timeout -k 10 500 python -u bench.py --no-coldstart --steps 1 --warmup 1 > gpurun_out/tune_r2k.log 2>&1 || { echo "tune failed"; tail -20 gpurun_out/tune_r2k.log; exit 1; }
diff dstack_amd/ops/tuned/gemm_tunableop_gfx950.csv gpurun_out/tune_r2k.csv
export DSTACK_AMD_GEMM_TUNING_FILE=gpurun_out/tune_r2k.csv
for i in 1 2; do
  for t in 0 1; do
    DSTACK_AMD_DGRAD_WT=$t timeout -k 10 300 python -u bench.py --no-coldstart --steps 6 > gpurun_out/ab_wt${t}_$i.log 2>&1 || { echo "bench t=$t failed"; tail -20 gpurun_out/ab_wt${t}_$i.log; exit 1; }
    echo "dgrad_wt=$t run=$i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_wt${t}_$i.log | tail -1) $(grep -o '"max_mem_gb": [0-9.]*' gpurun_out/ab_wt${t}_$i.log | tail -1)"
  done
done
bash tools/prof_tag.sh r2k
