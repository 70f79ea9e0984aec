set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
E2E_PROBE=1 E2E_STEPS=3 timeout -k 10 700 python -u tools/e2e_gpu_apply.py > gpurun_out/e2e_gpu_apply_probe_r1y.log 2>&1; rc=$?
tail -c 2500 gpurun_out/e2e_gpu_apply_probe_r1y.log; echo "rc=$rc"; exit $rc
