# Final check at HEAD: smoke, full GPU suite, default bench
# Final check at HEAD: smoke, full GPU suite, default bench
set -o pipefail
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r5g.log 2>&1
step pytest timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r5g.log 2>&1
tail -2 gpurun_out/pytest_r5g.log
step bench timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r5g.log 2>&1
tail -1 gpurun_out/bench_r5g.log | cut -c1-300
exit 0
