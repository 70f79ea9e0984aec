# skewed 8-wave forward (late waves one phase behind, 3-stage asm-DMA ring) vs lockstep forward
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q -k "variants_agree or flash" --timeout 200 --timeout-method thread > gpurun_out/attn_tests_r1zg.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/attn_tests_r1zg.log; exit 1; }
tail -1 gpurun_out/attn_tests_r1zg.log
for r in 1 2 3; do
  for sk in 1 0; do
    DSTACK_AMD_FA_FWD_SKEW=$sk timeout -k 10 120 python tools/bench_attn.py > gpurun_out/attn_skew${sk}_$r.json 2>gpurun_out/attn_skew${sk}_$r.err || { echo "bench failed skew=$sk"; tail -5 gpurun_out/attn_skew${sk}_$r.err; exit 1; }
    echo "skew=$sk run=$r $(cut -c1-120 gpurun_out/attn_skew${sk}_$r.json)"
  done
done
