# Serving refresh at HEAD (qkv-bias / family changes this round): Llama-3-8B bf16 and fp8 weights,
# 256 prompts x 1024 in / 256 out, 1 GPU
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench_serve.py --model llama-3-8b --num-prompts 256 --input-len 1024 --output-len 256 \
  > gpurun_out/serve_8b_r4z.log 2>&1 || { echo "8b bench failed"; tail -30 gpurun_out/serve_8b_r4z.log; exit 1; }
tail -1 gpurun_out/serve_8b_r4z.log | cut -c1-400
timeout -k 10 400 python -u bench_serve.py --model llama-3-8b --quantization fp8 --num-prompts 256 --input-len 1024 \
  --output-len 256 > gpurun_out/serve_8b_fp8_r4z.log 2>&1 || { echo "8b fp8 bench failed"; tail -30 gpurun_out/serve_8b_fp8_r4z.log; exit 1; }
tail -1 gpurun_out/serve_8b_fp8_r4z.log | cut -c1-400
