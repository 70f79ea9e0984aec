# fwd attention: prefetched S phase (PF=1, default) vs one-read-per-MFMA (PF=0), interleaved same-box runs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q -k "flash or attention" --timeout 120 --timeout-method thread > gpurun_out/attn_tests_r1ze.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/attn_tests_r1ze.log; exit 1; }
tail -1 gpurun_out/attn_tests_r1ze.log
for r in 1 2 3; do
  for pf in 1 0; do
    DSTACK_AMD_FA_FWD_PF=$pf timeout -k 10 120 python tools/bench_attn.py > gpurun_out/attn_pf${pf}_$r.json 2>/dev/null || { echo "bench failed pf=$pf"; exit 1; }
    echo "pf=$pf run=$r $(cat gpurun_out/attn_pf${pf}_$r.json)"
  done
done
