set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_ops_gpu.py -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"
timeout -k 10 300 python tools/bench_ops.py > gpurun_out/bench_ops.json 2> gpurun_out/bench_ops.err; echo "ops rc=$?"
timeout -k 10 400 python bench.py --steps 3 --warmup 2 > gpurun_out/bench_mb1.log 2>&1; echo "bench rc=$?"
timeout -k 10 400 python bench.py --steps 3 --warmup 2 --micro-batch 2 > gpurun_out/bench_mb2.log 2>&1; echo "bench rc=$?"
timeout -k 10 400 python bench.py --steps 3 --warmup 2 --grad-accum 2 > gpurun_out/bench_ga2.log 2>&1; echo "bench rc=$?"
