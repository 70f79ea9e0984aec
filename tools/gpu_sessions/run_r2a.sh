# round-2 start: smoke, all GPU tests, default bench (with cold start), kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r2a.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_r2a.log; exit 1; }
tail -1 gpurun_out/smoke_r2a.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r2a.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_r2a.log | head -10; exit 1; }
tail -1 gpurun_out/gpu_tests_r2a.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default_r2a.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_default_r2a.log; exit 1; }
tail -1 gpurun_out/bench_default_r2a.log | cut -c1-700
bash tools/prof_tag.sh r2a
