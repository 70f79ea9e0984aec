# driver-style round-end run at HEAD: smoke, full GPU suite, bench.py --gpus 1 --steps 20 --warmup 5
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r3k.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_r3k.log; exit 1; }
tail -1 gpurun_out/smoke_r3k.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r3k.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_r3k.log | head -10; exit 1; }
tail -1 gpurun_out/gpu_tests_r3k.log
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r3k.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_r3k.log; exit 1; }
tail -1 gpurun_out/bench_r3k.log | cut -c1-700
