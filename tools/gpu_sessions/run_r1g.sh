# delta tiled kernel + two-pass colsum: GPU tests, attention/ops microbench, headline bench, kernel stats
set -o pipefail
mkdir -p gpurun_out/prof_r1g
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r1g.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests_r1g.log; exit 1; }
tail -2 gpurun_out/gpu_tests_r1g.log
timeout -k 10 200 python -u tools/bench_attn.py > gpurun_out/attn_r1g.json 2>&1 || { echo "attn failed"; tail -20 gpurun_out/attn_r1g.json; exit 1; }
cat gpurun_out/attn_r1g.json
timeout -k 10 400 python -u bench.py --no-coldstart > gpurun_out/bench_r1g.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_r1g.log; exit 1; }
tail -1 gpurun_out/bench_r1g.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1g -o run -- python3 bench.py --steps 2 --warmup 1 --no-coldstart > gpurun_out/prof_bench_r1g.log 2>&1; echo "prof rc=$?"
