# A/B: attention backward -- HEAD~ build (.ab_old) vs current (row-constant init, dq 8 waves) vs current with dq 4 waves
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "flash or llama" > gpurun_out/gpu_tests_r1t.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests_r1t.log; exit 1; }
DSTACK_AMD_FA_DQ_WAVES=4 timeout -k 10 200 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "flash" >> gpurun_out/gpu_tests_r1t.log 2>&1 || { echo "tests(dq4) failed"; tail -30 gpurun_out/gpu_tests_r1t.log; exit 1; }
grep passed gpurun_out/gpu_tests_r1t.log
R=$GRAFT_REPO_ROOT
for i in 1 2 3; do
  (cd $R/.ab_old && timeout -k 10 200 python tools/bench_attn.py 2>/dev/null | grep -o '"bwd_ms": [0-9.]*' | sed "s/^/old /") || exit 1
  (cd $R && timeout -k 10 200 python tools/bench_attn.py 2>/dev/null | grep -o '"bwd_ms": [0-9.]*\|"bwd_rel_err": [0-9.e-]*' | tr '\n' ' ' | sed "s/^/new_dq8 /") || exit 1; echo
  (cd $R && DSTACK_AMD_FA_DQ_WAVES=4 timeout -k 10 200 python tools/bench_attn.py 2>/dev/null | grep -o '"bwd_ms": [0-9.]*' | sed "s/^/new_dq4 /") || exit 1
done
