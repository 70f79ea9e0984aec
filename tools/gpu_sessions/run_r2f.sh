# paged decode with the XCD-spread split grid + block-per-row RMSNorm: tests, microbench, 70B serving
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_serving.py tests/test_ops_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r2f.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error" gpurun_out/gpu_tests_r2f.log | head; tail -30 gpurun_out/gpu_tests_r2f.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r2f.log
timeout -k 10 300 python -u tools/bench_paged_decode.py > gpurun_out/bench_paged_decode_r2f.jsonl 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_paged_decode_r2f.jsonl; exit 1; }
timeout -k 10 500 python -u bench_serve.py --model llama-3-70b --num-prompts 256 --input-len 1024 --output-len 256 > gpurun_out/serve_70b_r2f.log 2>&1 || { echo "70b bench failed"; tail -30 gpurun_out/serve_70b_r2f.log; exit 1; }
tail -1 gpurun_out/serve_70b_r2f.log | cut -c1-900
timeout -k 10 300 python -u bench_serve.py --model llama-3-8b --num-prompts 256 --input-len 1024 --output-len 256 > gpurun_out/serve_8b_r2f.log 2>&1 || { echo "8b bench failed"; tail -30 gpurun_out/serve_8b_r2f.log; exit 1; }
tail -1 gpurun_out/serve_8b_r2f.log | cut -c1-900
