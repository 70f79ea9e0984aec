set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "transpose or wgrad or llama" > gpurun_out/gpu_tests_r1k.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests_r1k.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r1k.log
timeout -k 10 120 python -u tools/bench_transpose.py 2>&1 | grep -v amdgpu.ids
bash tools/prof_tag.sh r1k
