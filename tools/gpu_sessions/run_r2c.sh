# serving: pipelined paged-decode kernel (tests + 8B/70B benches), decode GEMM timing before/after
# TunableOp tuning of the decode shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export DSTACK_AMD_GEMM_TUNING_FILE=$GRAFT_REPO_ROOT/gpurun_out/gemm_tunableop_serving_gfx950.csv
timeout -k 10 300 python -u -m pytest tests/test_serving.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/serving_tests_r2c.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/serving_tests_r2c.log; exit 1; }
tail -1 gpurun_out/serving_tests_r2c.log
timeout -k 10 300 python -u bench_serve.py --model llama-3-8b --num-prompts 128 --input-len 512 --output-len 128 > gpurun_out/serve_8b_r2c.log 2>&1 || { echo "8b bench failed"; tail -30 gpurun_out/serve_8b_r2c.log; exit 1; }
tail -1 gpurun_out/serve_8b_r2c.log | cut -c1-900
timeout -k 10 200 python -u tools/tune_serving_gemms.py --mode off > gpurun_out/gemm_serving_off_r2c.jsonl 2>&1 || { echo "gemm timing failed"; tail -20 gpurun_out/gemm_serving_off_r2c.jsonl; exit 1; }
DSTACK_AMD_GEMM_TUNE_MS=100 timeout -k 10 600 python -u tools/tune_serving_gemms.py --mode tune > gpurun_out/gemm_serving_tune_r2c.jsonl 2>&1 || { echo "gemm tuning failed"; tail -20 gpurun_out/gemm_serving_tune_r2c.jsonl; exit 1; }
timeout -k 10 200 python -u tools/tune_serving_gemms.py --mode use > gpurun_out/gemm_serving_use_r2c.jsonl 2>&1 || { echo "gemm timing (tuned) failed"; tail -20 gpurun_out/gemm_serving_use_r2c.jsonl; exit 1; }
tail -1 gpurun_out/gemm_serving_use_r2c.jsonl
timeout -k 10 500 python -u bench_serve.py --model llama-3-70b --num-prompts 256 --input-len 1024 --output-len 256 > gpurun_out/serve_70b_r2c.log 2>&1 || { echo "70b bench failed"; tail -30 gpurun_out/serve_70b_r2c.log; exit 1; }
tail -1 gpurun_out/serve_70b_r2c.log | cut -c1-900
