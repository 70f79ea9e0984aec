set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u tools/e2e_gpu_apply.py > gpurun_out/e2e_gpu_apply_r1o.log 2>&1; rc=$?
tail -c 4000 gpurun_out/e2e_gpu_apply_r1o.log; echo "rc=$rc"; exit $rc
