# Round-4 evidence refresh at HEAD: smoke + GPU suite (agents changed), the dstack apply path on the GPU box (native shim/runner, the
# real bench as the job), then the serving engine on Llama-3-8B (bf16 and fp8 weights + fp8 KV)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
cd $R
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6b.log 2>&1
step pytest timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r6b.log 2>&1
tail -2 gpurun_out/pytest_r6b.log
step e2e timeout -k 10 500 python tools/e2e_gpu_apply.py > gpurun_out/e2e_gpu_apply_r6b.log 2>&1
tail -1 gpurun_out/e2e_gpu_apply_r6b.log | cut -c1-400
step serve8b timeout -k 10 400 python bench_serve.py --model llama-3-8b > gpurun_out/serve_8b_r6b.log 2>&1
tail -1 gpurun_out/serve_8b_r6b.log | cut -c1-400
step serve8b_fp8 timeout -k 10 400 python bench_serve.py --model llama-3-8b --quantization fp8 --kv-cache-dtype fp8 > gpurun_out/serve_8b_fp8kv_r6b.log 2>&1
tail -1 gpurun_out/serve_8b_fp8kv_r6b.log | cut -c1-400
exit 0
