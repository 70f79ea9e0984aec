# decode GEMV kernel (M <= 4): serving GPU tests, GEMV vs hipBLASLt microbench, 70B 32k-prompt latency A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_serving.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/serving_tests_r2o.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/serving_tests_r2o.log | head -20; exit 1; }
tail -1 gpurun_out/serving_tests_r2o.log
timeout -k 10 300 python -u tools/bench_gemv.py > gpurun_out/bench_gemv_r2o.log 2>&1 || { echo "gemv bench failed"; tail -20 gpurun_out/bench_gemv_r2o.log; exit 1; }
grep -v "^{" gpurun_out/bench_gemv_r2o.log | cut -c1-200
for g in 0 1; do
  DSTACK_AMD_GEMV=$g timeout -k 10 500 python -u bench_serve.py --model llama-3-70b --latency --input-len 32000 --output-len 128 --repeats 2 > gpurun_out/serve_70b_latency_gemv${g}_r2o.log 2>&1 || { echo "latency bench failed"; tail -30 gpurun_out/serve_70b_latency_gemv${g}_r2o.log; exit 1; }
  echo "gemv=$g $(grep -o '"e2e_p50_s": [0-9.]*\|"tpot_p50_ms": [0-9.]*\|"ttft_p50_s": [0-9.]*' gpurun_out/serve_70b_latency_gemv${g}_r2o.log | tr '\n' ' ')"
done
