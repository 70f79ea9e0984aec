# Round-4 final checkpoint at HEAD: smoke, full GPU suite, default bench, and a rocprofv3 kernel table of the step
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
cd $R
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6d.log 2>&1
step pytest timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r6d.log 2>&1
tail -2 gpurun_out/pytest_r6d.log
step bench timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r6d.log 2>&1
tail -1 gpurun_out/bench_r6d.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
step prof timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_step_r6d -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/prof_step_r6d.log 2>&1
exit 0
