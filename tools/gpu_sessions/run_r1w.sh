# A/B: attention kernels with builtin LDS-DMA (HEAD build in .ab_old) vs inline-asm LDS-DMA (tree)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "flash or llama" > gpurun_out/gpu_tests_r1w.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests_r1w.log; exit 1; }
grep passed gpurun_out/gpu_tests_r1w.log
R=$GRAFT_REPO_ROOT
for i in 1 2 3; do
  (cd $R/.ab_old && timeout -k 10 200 python tools/bench_attn.py 2>/dev/null | grep -o '"fwd_ms": [0-9.]*\|"bwd_ms": [0-9.]*' | tr '\n' ' ' | sed "s/^/old /") || exit 1; echo
  (cd $R && timeout -k 10 200 python tools/bench_attn.py 2>/dev/null | grep -o '"fwd_ms": [0-9.]*\|"bwd_ms": [0-9.]*\|"fwd_max_err": [0-9.e-]*\|"bwd_rel_err": [0-9.e-]*' | tr '\n' ' ' | sed "s/^/asm /") || exit 1; echo
done
