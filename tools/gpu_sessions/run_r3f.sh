# fp8 GEMV with 1 / 2 / 4 output rows per wave (x reuse; DSTACK_AMD_GEMV_FP8_R): correctness tests then interleaved timing
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2 4; do
  DSTACK_AMD_GEMV_FP8_R=$r timeout -k 10 300 python -u -m pytest tests/test_serving.py -m gpu -x -q --timeout 120 -k "gemv_fp8 or fp8_engine" > gpurun_out/gemv_fp8_tests_r$r.log 2>&1 || { echo "tests failed R=$r"; grep -E "FAIL|Error|assert" gpurun_out/gemv_fp8_tests_r$r.log | head; exit 1; }
  echo "R=$r $(tail -1 gpurun_out/gemv_fp8_tests_r$r.log)"
done
for rep in 1 2; do
  for r in 1 2 4; do
    DSTACK_AMD_GEMV_FP8_R=$r timeout -k 10 300 python -u tools/bench_gemv.py > gpurun_out/bench_gemv_fp8_R${r}_r3f_$rep.log 2>&1 || { echo "bench failed"; exit 1; }
    echo "rep $rep R=$r"; grep " 1 {" gpurun_out/bench_gemv_fp8_R${r}_r3f_$rep.log | sed 's/"gemv_ms.*"fp8_ms"/fp8_ms/' | cut -c1-110
  done
done
