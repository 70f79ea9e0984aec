# fp8 serving benchmarks with the tuned fp8 decode GEMMs + fp8 GPU tests + decode-step profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u bench_serve.py --model llama-3-70b --quantization fp8 --num-prompts 256 --input-len 1024 --output-len 256 > gpurun_out/serve_70b_fp8_r2z.log 2>&1 || { echo "70b fp8 failed"; tail -30 gpurun_out/serve_70b_fp8_r2z.log; exit 1; }
tail -1 gpurun_out/serve_70b_fp8_r2z.log | cut -c1-800
timeout -k 10 500 python -u bench_serve.py --model llama-3-70b --quantization fp8 --latency --input-len 32000 --output-len 128 --repeats 2 > gpurun_out/serve_70b_fp8_latency32k_r2z.log 2>&1 || { echo "latency failed"; tail -30 gpurun_out/serve_70b_fp8_latency32k_r2z.log; exit 1; }
tail -1 gpurun_out/serve_70b_fp8_latency32k_r2z.log | cut -c1-800
timeout -k 10 300 python -u bench_serve.py --model llama-3-8b --quantization fp8 --num-prompts 256 --input-len 1024 --output-len 256 > gpurun_out/serve_8b_fp8_r2z.log 2>&1 || { echo "8b fp8 failed"; tail -30 gpurun_out/serve_8b_fp8_r2z.log; exit 1; }
tail -1 gpurun_out/serve_8b_fp8_r2z.log | cut -c1-800
timeout -k 10 300 python -u -m pytest tests/test_serving.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/serving_tests_r2z.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/serving_tests_r2z.log | head -20; exit 1; }
tail -1 gpurun_out/serving_tests_r2z.log
mkdir -p gpurun_out/prof_r2z
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2z -o run -- python3 bench_serve.py --model llama-3-70b --quantization fp8 --num-prompts 256 --input-len 1024 --output-len 64 > gpurun_out/prof_serve_r2z.log 2>&1; echo "prof rc=$?"
python3 tools/step_breakdown.py gpurun_out/prof_r2z/run_kernel_trace.csv 20 > gpurun_out/decode_step_breakdown_70b_fp8_r2z.txt 2>&1; head -14 gpurun_out/decode_step_breakdown_70b_fp8_r2z.txt
