# amdsmi collector on the MI355X (xGMI / HBM fields), metrics + health GPU tests, serving families on HIP
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 native/build/dstack-shim --gpu-metrics > gpurun_out/gpu_metrics_r4t.json 2>&1; echo "metrics rc=$?"
head -c 800 gpurun_out/gpu_metrics_r4t.json; echo
timeout -k 10 400 python -u -m pytest tests/test_gpu_metrics.py tests/test_gpu_health.py "tests/test_serving.py::test_gpu_engine_matches_cpu_and_graphs" -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_r4t.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r4t.log; exit $rc
