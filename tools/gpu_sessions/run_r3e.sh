# tune the fp8 prefill GEMMs (M = 16384 packed prompt tokens, 32000 single long prompt) of Llama-3-70B/8B,
# then re-run the 70B fp8 throughput and 32k latency benchmarks with them
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export DSTACK_AMD_GEMM_TUNE_MS=100
DSTACK_AMD_GEMM_TUNING_FILE=$GRAFT_REPO_ROOT/gpurun_out/serving_fp8_prefill_tuned.csv timeout -k 10 900 python -u tools/tune_serving_gemms.py --dtype fp8 --mode tune --models llama-3-70b,llama-3-8b --buckets 16384,32000 > gpurun_out/tune_fp8_prefill_r3e.jsonl 2>&1 || { echo "tune failed"; tail -20 gpurun_out/tune_fp8_prefill_r3e.jsonl; exit 1; }
grep -v Validator gpurun_out/serving_fp8_prefill_tuned.csv >> dstack_amd/ops/tuned/gemm_tunableop_serving_gfx950.csv
grep '"M": 16384' gpurun_out/tune_fp8_prefill_r3e.jsonl | cut -c1-200
timeout -k 10 500 python -u bench_serve.py --model llama-3-70b --quantization fp8 --kv-cache-dtype fp8 --num-prompts 256 --input-len 1024 --output-len 256 > gpurun_out/serve_70b_fp8kv_r3e.log 2>&1 || { echo "70b failed"; tail -30 gpurun_out/serve_70b_fp8kv_r3e.log; exit 1; }
tail -1 gpurun_out/serve_70b_fp8kv_r3e.log | cut -c1-700
timeout -k 10 500 python -u bench_serve.py --model llama-3-70b --quantization fp8 --kv-cache-dtype fp8 --latency --input-len 32000 --output-len 128 --repeats 2 > gpurun_out/serve_70b_fp8kv_latency32k_r3e.log 2>&1 || { echo "latency failed"; tail -30 gpurun_out/serve_70b_fp8kv_latency32k_r3e.log; exit 1; }
tail -1 gpurun_out/serve_70b_fp8kv_latency32k_r3e.log | cut -c1-700
