# continue GEMM tuning (remaining backward shapes) with a shorter per-candidate budget
set -o pipefail
mkdir -p gpurun_out
(while true; do sleep 50; date >> gpurun_out/heartbeat.txt; done) &
HB=$!
trap "kill $HB" EXIT
cp dstack_amd/ops/tuned/gemm_tunableop_gfx950.csv gpurun_out/gemm_tunableop_gfx950.csv
export DSTACK_AMD_GEMM_TUNE_MS=8 DSTACK_AMD_GEMM_TUNE_ITERS=4
export DSTACK_AMD_GEMM_TUNING_FILE=$GRAFT_REPO_ROOT/gpurun_out/gemm_tunableop_gfx950.csv
DSTACK_AMD_GEMM_TUNING=tune timeout -k 10 1050 python bench.py --steps 1 --warmup 1 --grad-accum 1 --no-coldstart > gpurun_out/tune2.log 2>&1
echo "tune rc=$?"
wc -l gpurun_out/gemm_tunableop_gfx950.csv
