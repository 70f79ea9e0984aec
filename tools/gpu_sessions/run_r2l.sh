# gradient accumulation depth: 2 vs 4 vs 8 micro-batches of 8192 tokens per optimizer step (same box)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
  for ga in 2 4 8; do
    timeout -k 10 400 python -u bench.py --no-coldstart --steps 4 --warmup 2 --grad-accum $ga > gpurun_out/ab_ga${ga}_$i.log 2>&1 || { echo "bench ga=$ga failed"; tail -20 gpurun_out/ab_ga${ga}_$i.log; exit 1; }
    echo "grad_accum=$ga run=$i $(grep -o '"value": [0-9.]*' gpurun_out/ab_ga${ga}_$i.log | tail -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_ga${ga}_$i.log | tail -1)"
  done
done
