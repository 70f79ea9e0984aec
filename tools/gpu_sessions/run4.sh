# smoke + GPU tests + probe + default bench (incl. cold start) + rocprof kernel stats
set -o pipefail
mkdir -p gpurun_out/prof4
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step smoke timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
step pytest timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
step probe timeout -k 10 120 native/build/dstack-probe --json > gpurun_out/probe.json 2> gpurun_out/probe.err
step bench timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step prof timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof4 -o run -- python3 bench.py --steps 2 --warmup 1 --no-coldstart > gpurun_out/prof4_bench.log 2>&1
find gpurun_out/prof4 -name "*stats*"
