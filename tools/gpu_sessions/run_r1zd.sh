set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python tools/diag/overlap_losses.py 2>&1 | grep -v amdgpu.ids | head -4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r1zd.log 2>&1 || { echo "tests failed"; grep -E "Error|assert" gpurun_out/gpu_tests_r1zd.log | head -10; exit 1; }
tail -1 gpurun_out/gpu_tests_r1zd.log
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/dist_gpu_check.py > gpurun_out/dist_gpu_check_r1zd.log 2>&1 || { tail -5 gpurun_out/dist_gpu_check_r1zd.log; exit 1; }
grep '^{' gpurun_out/dist_gpu_check_r1zd.log
bash tools/prof_tag.sh r1zd
