# fp8 serving benchmarks: Llama-3-70B / 8B throughput (256 x 1024 in / 256 out) and 70B single 32k prompt
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u bench_serve.py --model llama-3-70b --quantization fp8 --num-prompts 256 --input-len 1024 --output-len 256 > gpurun_out/serve_70b_fp8_r2w.log 2>&1 || { echo "70b fp8 failed"; tail -30 gpurun_out/serve_70b_fp8_r2w.log; exit 1; }
tail -1 gpurun_out/serve_70b_fp8_r2w.log | cut -c1-800
timeout -k 10 500 python -u bench_serve.py --model llama-3-70b --quantization fp8 --latency --input-len 32000 --output-len 128 --repeats 2 > gpurun_out/serve_70b_fp8_latency32k_r2w.log 2>&1 || { echo "latency failed"; tail -30 gpurun_out/serve_70b_fp8_latency32k_r2w.log; exit 1; }
tail -1 gpurun_out/serve_70b_fp8_latency32k_r2w.log | cut -c1-800
timeout -k 10 300 python -u bench_serve.py --model llama-3-8b --quantization fp8 --num-prompts 256 --input-len 1024 --output-len 256 > gpurun_out/serve_8b_fp8_r2w.log 2>&1 || { echo "8b fp8 failed"; tail -30 gpurun_out/serve_8b_fp8_r2w.log; exit 1; }
tail -1 gpurun_out/serve_8b_fp8_r2w.log | cut -c1-800
