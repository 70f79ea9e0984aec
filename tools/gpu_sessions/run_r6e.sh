# Serving refresh at HEAD on Llama-3-70B, one MI355X: bf16, and fp8 weights + fp8 KV cache
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
cd $R
step serve70b timeout -k 10 500 python -u bench_serve.py --model llama-3-70b > gpurun_out/serve_70b_r6e.log 2>&1
tail -1 gpurun_out/serve_70b_r6e.log | cut -c1-300
step serve70b_fp8kv timeout -k 10 500 python -u bench_serve.py --model llama-3-70b --quantization fp8 --kv-cache-dtype fp8 > gpurun_out/serve_70b_fp8kv_r6e.log 2>&1
tail -1 gpurun_out/serve_70b_fp8kv_r6e.log | cut -c1-300
exit 0
