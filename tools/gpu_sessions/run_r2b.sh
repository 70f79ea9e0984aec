# serving engine first GPU contact: serving GPU tests (kernels vs fp32 refs, graphs), then a short
# 8B throughput bench and a 70B throughput bench with a kernel profile of the 8B run
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_serving.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/serving_tests_r2b.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/serving_tests_r2b.log | head -20; tail -30 gpurun_out/serving_tests_r2b.log; exit 1; }
tail -1 gpurun_out/serving_tests_r2b.log
timeout -k 10 300 python -u bench_serve.py --model llama-3-8b --num-prompts 128 --input-len 512 --output-len 128 > gpurun_out/serve_8b_r2b.log 2>&1 || { echo "8b bench failed"; tail -30 gpurun_out/serve_8b_r2b.log; exit 1; }
tail -1 gpurun_out/serve_8b_r2b.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_serve_r2b -o run -- python3 bench_serve.py --model llama-3-8b --num-prompts 64 --input-len 512 --output-len 64 > gpurun_out/prof_serve_r2b.log 2>&1; echo "prof rc=$?"
timeout -k 10 500 python -u bench_serve.py --model llama-3-70b --num-prompts 256 --input-len 1024 --output-len 256 > gpurun_out/serve_70b_r2b.log 2>&1 || { echo "70b bench failed"; tail -30 gpurun_out/serve_70b_r2b.log; exit 1; }
tail -1 gpurun_out/serve_70b_r2b.log
