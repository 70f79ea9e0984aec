# GEMM tuning (TunableOp/hipBLASLt) for the Llama-3-8B training shapes, then A/B bench
set -o pipefail
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
(while true; do sleep 50; date >> gpurun_out/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
export DSTACK_AMD_GEMM_TUNE_MS=30 DSTACK_AMD_GEMM_TUNE_ITERS=20
export DSTACK_AMD_GEMM_TUNING_FILE=$GRAFT_REPO_ROOT/gpurun_out/gemm_tunableop_gfx950.csv
step tune env DSTACK_AMD_GEMM_TUNING=tune timeout -k 10 900 python bench.py --steps 1 --warmup 1 --grad-accum 1 --no-coldstart > gpurun_out/tune.log 2>&1
ls -la gpurun_out/gemm_tunableop_gfx950.csv
step use env DSTACK_AMD_GEMM_TUNING=use timeout -k 10 400 python bench.py --no-coldstart > gpurun_out/bench_tuned.log 2>&1
step off env DSTACK_AMD_GEMM_TUNING=off timeout -k 10 400 python bench.py --no-coldstart > gpurun_out/bench_untuned.log 2>&1
tail -1 gpurun_out/bench_tuned.log gpurun_out/bench_untuned.log
