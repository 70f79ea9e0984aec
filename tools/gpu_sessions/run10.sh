# 8-wave dK/dV default: GPU suite, bench, profile
set -o pipefail
mkdir -p gpurun_out/prof10
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest10.log 2>&1
step bench timeout -k 10 600 python bench.py > gpurun_out/bench10.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step prof timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof10 -o run -- python3 bench.py --steps 2 --warmup 1 --no-coldstart > gpurun_out/prof10_bench.log 2>&1
tail -1 gpurun_out/bench10.log
