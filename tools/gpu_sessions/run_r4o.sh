# Round-3 bench at HEAD (driver-style) + rocprofv3 kernel statistics of a short bench
set -o pipefail
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step bench timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r4o.log 2>&1
tail -1 gpurun_out/bench_r4o.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step prof timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4o -o run -- python bench.py --steps 3 --warmup 2 --no-coldstart > gpurun_out/prof_r4o.log 2>&1
ls gpurun_out/prof_r4o | head
exit 0
