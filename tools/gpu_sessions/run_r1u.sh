set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r1u.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests_r1u.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r1u.log
timeout -k 10 120 python -u __graft_entry__.py smoke 2>&1 | grep -v amdgpu.ids
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r1u.log 2>&1 || { tail -20 gpurun_out/bench_r1u.log; exit 1; }
tail -1 gpurun_out/bench_r1u.log | cut -c1-400
