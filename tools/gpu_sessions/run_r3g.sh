# fp8 GEMV with rows-per-wave chosen by N: serving GPU tests, 70B fp8 single 32k prompt latency, 8B fp8 throughput
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_serving.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/serving_tests_r3g.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/serving_tests_r3g.log | head -20; exit 1; }
tail -1 gpurun_out/serving_tests_r3g.log
timeout -k 10 500 python -u bench_serve.py --model llama-3-70b --quantization fp8 --kv-cache-dtype fp8 --latency --input-len 32000 --output-len 128 --repeats 2 > gpurun_out/serve_70b_fp8kv_latency32k_r3g.log 2>&1 || { echo "latency failed"; tail -30 gpurun_out/serve_70b_fp8kv_latency32k_r3g.log; exit 1; }
tail -1 gpurun_out/serve_70b_fp8kv_latency32k_r3g.log | cut -c1-700
