# fp8 KV cache: serving GPU tests, then 70B (fp8 weights + fp8 KV) throughput and 32k latency, 8B throughput,
# and the 70B decode-step profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_serving.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/serving_tests_r3a.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/serving_tests_r3a.log | head -20; exit 1; }
tail -1 gpurun_out/serving_tests_r3a.log
timeout -k 10 500 python -u bench_serve.py --model llama-3-70b --quantization fp8 --kv-cache-dtype fp8 --num-prompts 256 --input-len 1024 --output-len 256 > gpurun_out/serve_70b_fp8kv_r3a.log 2>&1 || { echo "70b failed"; tail -30 gpurun_out/serve_70b_fp8kv_r3a.log; exit 1; }
tail -1 gpurun_out/serve_70b_fp8kv_r3a.log | cut -c1-900
timeout -k 10 500 python -u bench_serve.py --model llama-3-70b --quantization fp8 --kv-cache-dtype fp8 --latency --input-len 32000 --output-len 128 --repeats 2 > gpurun_out/serve_70b_fp8kv_latency32k_r3a.log 2>&1 || { echo "latency failed"; tail -30 gpurun_out/serve_70b_fp8kv_latency32k_r3a.log; exit 1; }
tail -1 gpurun_out/serve_70b_fp8kv_latency32k_r3a.log | cut -c1-700
timeout -k 10 300 python -u bench_serve.py --model llama-3-8b --quantization fp8 --kv-cache-dtype fp8 --num-prompts 256 --input-len 1024 --output-len 256 > gpurun_out/serve_8b_fp8kv_r3a.log 2>&1 || { echo "8b failed"; tail -30 gpurun_out/serve_8b_fp8kv_r3a.log; exit 1; }
tail -1 gpurun_out/serve_8b_fp8kv_r3a.log | cut -c1-700
mkdir -p gpurun_out/prof_r3a
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3a -o run -- python3 bench_serve.py --model llama-3-70b --quantization fp8 --kv-cache-dtype fp8 --num-prompts 256 --input-len 1024 --output-len 64 > gpurun_out/prof_serve_r3a.log 2>&1; echo "prof rc=$?"
python3 tools/step_breakdown.py gpurun_out/prof_r3a/run_kernel_trace.csv 20 > gpurun_out/decode_step_breakdown_70b_fp8kv_r3a.txt 2>&1; head -14 gpurun_out/decode_step_breakdown_70b_fp8kv_r3a.txt
