# token-contiguous wgrad operands: GPU tests, in-situ TunableOp pass for the new layouts, A/B bench
set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r1i.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests_r1i.log; exit 1; }
tail -2 gpurun_out/gpu_tests_r1i.log
cp dstack_amd/ops/tuned/gemm_tunableop_gfx950.csv gpurun_out/tune_r1i.csv
DSTACK_AMD_GEMM_TUNING=tune DSTACK_AMD_GEMM_TUNING_FILE=$PWD/gpurun_out/tune_r1i.csv timeout -k 10 500 python -u bench.py --steps 1 --warmup 1 --no-coldstart > gpurun_out/tune_r1i.log 2>&1 || { echo "tune failed"; tail -20 gpurun_out/tune_r1i.log; exit 1; }
wc -l gpurun_out/tune_r1i.csv
for v in a b; do
DSTACK_AMD_GEMM_TUNING_FILE=$PWD/gpurun_out/tune_r1i.csv timeout -k 10 300 python -u bench.py --no-coldstart > gpurun_out/bench_r1i_tuned_$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_r1i_tuned_$v.log; exit 1; }
echo "tuned: $(tail -1 gpurun_out/bench_r1i_tuned_$v.log | cut -c1-260)"
DSTACK_AMD_WGRAD=strided timeout -k 10 300 python -u bench.py --no-coldstart > gpurun_out/bench_r1i_strided_$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_r1i_strided_$v.log; exit 1; }
echo "strided: $(tail -1 gpurun_out/bench_r1i_strided_$v.log | cut -c1-260)"
done
