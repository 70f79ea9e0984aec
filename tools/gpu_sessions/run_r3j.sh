# re-tune the training GEMMs from scratch with a longer budget per shape (1 s, 200 iterations), then
# A/B the bench with the shipped CSV vs the re-tuned one (interleaved, same box)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
NEW=$GRAFT_REPO_ROOT/gpurun_out/train_retune_r3j.csv
DSTACK_AMD_GEMM_TUNING=tune DSTACK_AMD_GEMM_TUNING_FILE=$NEW DSTACK_AMD_GEMM_TUNE_MS=1000 DSTACK_AMD_GEMM_TUNE_ITERS=200 \
  timeout -k 10 900 python -u bench.py --steps 1 --warmup 1 --no-coldstart > gpurun_out/retune_r3j.log 2>&1 || { echo "retune failed"; tail -20 gpurun_out/retune_r3j.log; exit 1; }
grep -c "" $NEW
for rep in 1 2; do
  for f in old new; do
    if [ $f = new ]; then export DSTACK_AMD_GEMM_TUNING_FILE=$NEW; else unset DSTACK_AMD_GEMM_TUNING_FILE; fi
    timeout -k 10 400 python -u bench.py --steps 4 --warmup 2 --no-coldstart > gpurun_out/bench_tune_${f}_r3j_$rep.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_tune_${f}_r3j_$rep.log; exit 1; }
    echo "rep $rep $f $(tail -1 gpurun_out/bench_tune_${f}_r3j_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/retune_ab_r3j.txt
  done
done
