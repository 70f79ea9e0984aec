set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/dist_gpu_check.py > gpurun_out/dist_gpu_check_r1m.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/dist_gpu_check_r1m.log | tail -20; echo "rc=$rc"; exit $rc
