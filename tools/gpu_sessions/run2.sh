set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_ops_gpu.py -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"
timeout -k 10 300 python tools/bench_ops.py > gpurun_out/bench_ops.json 2> gpurun_out/bench_ops.err; echo "ops rc=$?"
timeout -k 10 400 python bench.py --steps 3 --warmup 2 > gpurun_out/bench_hip.log 2>&1; echo "bench rc=$?"
