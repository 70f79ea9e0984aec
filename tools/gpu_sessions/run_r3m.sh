# after the native JSON changes: the bench task through the server on the GPU, and bench.py's cold start
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/e2e_gpu_apply.py > gpurun_out/e2e_gpu_apply_r3m.log 2>&1 || { echo "e2e failed"; tail -30 gpurun_out/e2e_gpu_apply_r3m.log; exit 1; }
tail -1 gpurun_out/e2e_gpu_apply_r3m.log | cut -c1-400
timeout -k 10 600 python -u bench.py --steps 3 --warmup 2 > gpurun_out/bench_r3m.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_r3m.log; exit 1; }
tail -1 gpurun_out/bench_r3m.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["cold_start_p50_s"], d["cold_start"])'
