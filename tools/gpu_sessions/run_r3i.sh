# fused add+RMSNorm -> fp8: serving GPU tests, then 70B fp8 throughput with the fusion off / on (interleaved)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_serving.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/serving_tests_r3i.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/serving_tests_r3i.log | head -20; exit 1; }
tail -1 gpurun_out/serving_tests_r3i.log
for f in 0 1 0 1; do
  DSTACK_AMD_FP8_FUSE_NORM=$f timeout -k 10 400 python -u bench_serve.py --model llama-3-70b --quantization fp8 --kv-cache-dtype fp8 --num-prompts 256 --input-len 1024 --output-len 256 > gpurun_out/serve_70b_fuse${f}_r3i.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/serve_70b_fuse${f}_r3i.log; exit 1; }
  echo "fuse=$f $(tail -1 gpurun_out/serve_70b_fuse${f}_r3i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["decode_tokens_per_s"], d["prefill_tokens_per_s"])')" | tee -a gpurun_out/fuse_norm_ab_r3i.txt
done
