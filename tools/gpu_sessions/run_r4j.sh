# Bench loss curve on the synthetic LM stream (fresh batch every micro-step): 5 warmup + 25 timed
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python bench.py --steps 25 --warmup 5 --no-coldstart > gpurun_out/bench_lm_r4j.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_lm_r4j.log; exit $rc
