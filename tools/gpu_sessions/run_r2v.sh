# fp8 serving: scaled_mm probe, fp8 kernel + engine tests, 70B fp8 vs bf16 throughput and batch-1 latency
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/probe_fp8_gemm.py > gpurun_out/probe_fp8_gemm_r2v.jsonl 2>&1 || { echo "probe failed"; tail -20 gpurun_out/probe_fp8_gemm_r2v.jsonl; exit 1; }
grep '^{' gpurun_out/probe_fp8_gemm_r2v.jsonl | cut -c1-400
timeout -k 10 400 python -u -m pytest tests/test_serving.py -m gpu -x -v --timeout 200 --timeout-method thread -k "fp8" > gpurun_out/fp8_tests_r2v.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/fp8_tests_r2v.log | head -20; exit 1; }
tail -1 gpurun_out/fp8_tests_r2v.log
