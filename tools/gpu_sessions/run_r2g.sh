# session re-entry (rebuilt tree): smoke, all GPU tests, default bench, attention + op microbenchmarks, kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r2g.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_r2g.log; exit 1; }
tail -1 gpurun_out/smoke_r2g.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r2g.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_r2g.log | head -10; exit 1; }
tail -1 gpurun_out/gpu_tests_r2g.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default_r2g.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_default_r2g.log; exit 1; }
tail -1 gpurun_out/bench_default_r2g.log | cut -c1-500
timeout -k 10 200 python -u tools/bench_attn.py > gpurun_out/bench_attn_r2g.log 2>&1 || { echo "attn bench failed"; tail -20 gpurun_out/bench_attn_r2g.log; exit 1; }
tail -3 gpurun_out/bench_attn_r2g.log
timeout -k 10 200 python -u tools/bench_transpose.py > gpurun_out/bench_transpose_r2g.log 2>&1 || { echo "transpose bench failed"; exit 1; }
cat gpurun_out/bench_transpose_r2g.log
bash tools/prof_tag.sh r2g
