# round-end style validation at HEAD: smoke, every GPU test, 2-rank ZeRO check on one GPU, default bench with cold start, kernel profile, task through the server on the GPU
# smoke, every GPU test, default bench with cold start, kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r3d.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_r3d.log; exit 1; }
tail -1 gpurun_out/smoke_r3d.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r3d.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests_r3d.log | head -10; exit 1; }
tail -1 gpurun_out/gpu_tests_r3d.log
timeout -k 10 300 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/dist_gpu_check.py > gpurun_out/dist_gpu_check_r3d.log 2>&1 || { echo "dist check failed"; tail -20 gpurun_out/dist_gpu_check_r3d.log; exit 1; }
grep '^{' gpurun_out/dist_gpu_check_r3d.log | tail -1 | cut -c1-600
timeout -k 10 600 python -u bench.py --steps 6 --warmup 2 > gpurun_out/bench_default_r3d.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_default_r3d.log; exit 1; }
tail -1 gpurun_out/bench_default_r3d.log | cut -c1-900
mkdir -p gpurun_out/prof_r3d
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3d -o run -- python3 bench.py --steps 1 --warmup 1 --no-coldstart > gpurun_out/prof_bench_r3d.log 2>&1; echo "prof rc=$?"
timeout -k 10 400 python -u tools/e2e_gpu_apply.py > gpurun_out/e2e_gpu_apply_r3d.log 2>&1; echo "e2e rc=$?"
tail -3 gpurun_out/e2e_gpu_apply_r3d.log | cut -c1-600
