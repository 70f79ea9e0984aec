# End-of-session checkpoint at HEAD: default bench (driver contract) and a rocprofv3 kernel table of
# the training step
set -o pipefail
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step bench timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r5e.log 2>&1
tail -1 gpurun_out/bench_r5e.log | cut -c1-400
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
step prof timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_step_r5e -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/prof_step_r5e.log 2>&1
exit 0
