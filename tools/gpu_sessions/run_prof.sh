set -o pipefail
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof_bench.log 2>&1; echo "prof rc=$?"
find gpurun_out/prof -name "*stats*" | head
