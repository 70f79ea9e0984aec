# Checkpoint at HEAD: smoke, full GPU suite, default bench, the e2e apply path (native shim/runner
# with the runner-reported port) on the GPU box
set -o pipefail
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r4w.log 2>&1
step pytest timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r4w.log 2>&1
tail -2 gpurun_out/pytest_r4w.log
step bench timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r4w.log 2>&1
tail -1 gpurun_out/bench_r4w.log | cut -c1-300
step e2e timeout -k 10 400 python tools/e2e_gpu_apply.py > gpurun_out/e2e_gpu_apply_r4w.log 2>&1
tail -1 gpurun_out/e2e_gpu_apply_r4w.log | cut -c1-400
exit 0
