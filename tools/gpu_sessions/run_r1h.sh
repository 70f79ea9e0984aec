set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
true
TUNE=1 timeout -k 10 600 python -u tools/bench_wgrad_layouts.py > gpurun_out/wgrad_layouts_tune.log 2>&1 || { tail -20 gpurun_out/wgrad_layouts_tune.log; exit 1; }
grep -v "^{" gpurun_out/wgrad_layouts_use.log; grep -v "^{" gpurun_out/wgrad_layouts_tune.log
cp /tmp/wgrad_layouts_tune.csv gpurun_out/ || true
