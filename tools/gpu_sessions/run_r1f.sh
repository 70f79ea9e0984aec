# Round-1 re-entry check: GPU tests, headline bench, rocprof kernel stats at HEAD
set -o pipefail
mkdir -p gpurun_out/prof_r1f
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r1f.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/gpu_tests_r1f.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r1f.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_r1f.log; exit 1; }
tail -1 gpurun_out/bench_r1f.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1f -o run -- python3 bench.py --steps 2 --warmup 1 --no-coldstart > gpurun_out/prof_bench_r1f.log 2>&1; echo "prof rc=$?"
