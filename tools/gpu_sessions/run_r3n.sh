# after the stop/fleet-delete locking changes: the bench task through the server on the GPU, plus a
# kernel-time profile of the training step at HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_r3n
timeout -k 10 400 python -u tools/e2e_gpu_apply.py > gpurun_out/e2e_gpu_apply_r3n.log 2>&1 || { echo "e2e failed"; tail -30 gpurun_out/e2e_gpu_apply_r3n.log; exit 1; }
tail -1 gpurun_out/e2e_gpu_apply_r3n.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3n -o run -- python3 bench.py --steps 2 --warmup 1 --no-coldstart > gpurun_out/prof_r3n_bench.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_r3n_bench.log; exit 1; }
echo "prof ok"
