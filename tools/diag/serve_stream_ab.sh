set -o pipefail
# Serving A/B of the weight-streaming decode fp8 GEMM (DSTACK_AMD_FP8_STREAM 0/1, interleaved) on the
# Llama-3-70B fp8 bench, after its GPU tests; logs under gpurun_out/r9u/
mkdir -p gpurun_out/r9u
bash tools/gpu_session.sh r9u test=fp8_stream || exit 1
A="--model llama-3-70b --quantization fp8 --kv-cache-dtype fp8"
i=0
for v in 0 1 0 1; do
  i=$((i + 1))
  DSTACK_AMD_FP8_STREAM=$v timeout -k 10 400 python -u bench_serve.py $A > gpurun_out/r9u/serve_stream$v.run$i.log 2>&1 || exit 1
  echo "serve stream=$v done"
done
