# A/B: flash-attention forward with 4 waves x 2 workgroups/CU vs 8 waves x 1 workgroup/CU
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
DSTACK_AMD_FA_FWD_WAVES=8 timeout -k 10 200 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "flash or llama" > gpurun_out/gpu_tests_r1s.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests_r1s.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r1s.log
for i in 1 2 3; do
  timeout -k 10 200 python tools/bench_attn.py 2>/dev/null | grep -o '"fwd_ms": [0-9.]*, "fwd_tflops": [0-9.]*' | sed "s/^/w4 /" || exit 1
  DSTACK_AMD_FA_FWD_WAVES=8 timeout -k 10 200 python tools/bench_attn.py 2>/dev/null | grep -o '"fwd_ms": [0-9.]*, "fwd_tflops": [0-9.]*, "bwd_ms": [0-9.]*\|"fwd_max_err": [0-9.e-]*' | tr '\n' ' ' | sed "s/^/w8 /" || exit 1
  echo
done
