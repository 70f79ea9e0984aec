# tune the fp8 (row-wise scaled) decode GEMMs of Llama-3-70B and -8B with TunableOp into
# gpurun_out/serving_fp8_tuned.csv (merged into dstack_amd/ops/tuned/ afterwards), then time them with the result
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export DSTACK_AMD_GEMM_TUNING_FILE=$GRAFT_REPO_ROOT/gpurun_out/serving_fp8_tuned.csv DSTACK_AMD_GEMM_TUNE_MS=100
timeout -k 10 900 python -u tools/tune_serving_gemms.py --dtype fp8 --mode tune --models llama-3-70b,llama-3-8b > gpurun_out/tune_fp8_r2y.jsonl 2>&1 || { echo "tune failed"; tail -20 gpurun_out/tune_fp8_r2y.jsonl; exit 1; }
wc -l gpurun_out/serving_fp8_tuned.csv
timeout -k 10 200 python -u tools/tune_serving_gemms.py --dtype fp8 --mode use --models llama-3-70b > gpurun_out/use_fp8_r2y.jsonl 2>&1 || { echo "use failed"; tail -20 gpurun_out/use_fp8_r2y.jsonl; exit 1; }
grep '"M": 256' gpurun_out/use_fp8_r2y.jsonl | cut -c1-300
