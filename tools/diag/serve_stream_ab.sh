set -o pipefail
# Serving A/B of the weight-streaming decode fp8 GEMM on the Llama-3-70B fp8 bench, interleaved, after
# its GPU tests: bash tools/diag/serve_stream_ab.sh <tag> <ENV=a> <ENV=b>  (default: the GEMM off / on);
# logs under gpurun_out/<tag>/
TAG=${1:-r9u}
A_ENV=${2:-DSTACK_AMD_FP8_STREAM=0}
B_ENV=${3:-DSTACK_AMD_FP8_STREAM=1}
mkdir -p "gpurun_out/$TAG"
bash tools/gpu_session.sh "$TAG" test=fp8_stream || exit 1
A="--model llama-3-70b --quantization fp8 --kv-cache-dtype fp8"
i=0
for e in "$A_ENV" "$B_ENV" "$A_ENV" "$B_ENV"; do
  i=$((i + 1))
  env "$e" timeout -k 10 400 python -u bench_serve.py $A > "gpurun_out/$TAG/serve.$e.run$i.log" 2>&1 || exit 1
  echo "serve $e done"
done
