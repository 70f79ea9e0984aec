set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r1zb.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_r1zb.log | head -20; tail -5 gpurun_out/gpu_tests_r1zb.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r1zb.log
bash tools/prof_tag.sh r1zb
