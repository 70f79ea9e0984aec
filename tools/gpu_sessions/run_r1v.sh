set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
E2E_TORCHRUN=1 timeout -k 10 700 python -u tools/e2e_gpu_apply.py > gpurun_out/e2e_gpu_apply_torchrun_r1v.log 2>&1; rc=$?
tail -c 3000 gpurun_out/e2e_gpu_apply_torchrun_r1v.log; echo "rc=$rc"; exit $rc
