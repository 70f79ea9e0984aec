# token-shard loader on the GPU (pinned ring + async H2D, train step on shard input)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_tokens_loader.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_tokens_r4v.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_tokens_r4v.log; exit $rc
