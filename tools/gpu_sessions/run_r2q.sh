# parallel split-KV combine + batch-1 GEMV: serving GPU tests, paged-decode microbench, 70B 32k latency,
# 70B/8B throughput
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_serving.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/serving_tests_r2q.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/serving_tests_r2q.log | head -20; exit 1; }
tail -1 gpurun_out/serving_tests_r2q.log
timeout -k 10 300 python -u tools/bench_paged_decode.py > gpurun_out/bench_paged_decode_r2q.jsonl 2>&1 || { echo "paged bench failed"; tail -20 gpurun_out/bench_paged_decode_r2q.jsonl; exit 1; }
tail -4 gpurun_out/bench_paged_decode_r2q.jsonl | cut -c1-300
timeout -k 10 500 python -u bench_serve.py --model llama-3-70b --latency --input-len 32000 --output-len 128 --repeats 2 > gpurun_out/serve_70b_latency32k_r2q.log 2>&1 || { echo "latency bench failed"; tail -30 gpurun_out/serve_70b_latency32k_r2q.log; exit 1; }
tail -1 gpurun_out/serve_70b_latency32k_r2q.log | cut -c1-700
timeout -k 10 500 python -u bench_serve.py --model llama-3-70b --num-prompts 256 --input-len 1024 --output-len 256 > gpurun_out/serve_70b_r2q.log 2>&1 || { echo "70b bench failed"; tail -30 gpurun_out/serve_70b_r2q.log; exit 1; }
tail -1 gpurun_out/serve_70b_r2q.log | cut -c1-700
timeout -k 10 300 python -u bench_serve.py --model llama-3-8b --num-prompts 256 --input-len 1024 --output-len 256 > gpurun_out/serve_8b_r2q.log 2>&1 || { echo "8b bench failed"; tail -30 gpurun_out/serve_8b_r2q.log; exit 1; }
tail -1 gpurun_out/serve_8b_r2q.log | cut -c1-700
