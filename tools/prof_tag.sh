# usage: bash tools/prof_tag.sh TAG  -> bench line + rocprofv3 kernel stats/trace under gpurun_out/prof_TAG
set -o pipefail
TAG=$1
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 300 python -u bench.py --no-coldstart > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 2 --warmup 1 --no-coldstart > gpurun_out/prof_bench_$TAG.log 2>&1; echo "prof rc=$?"
