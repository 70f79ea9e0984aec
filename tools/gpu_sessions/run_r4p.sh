# A/B: micro-batch 2 x grad-accum 4 vs micro-batch 1 x grad-accum 8 (same 64k tokens/step), interleaved
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_mb_r4p.txt
for rep in 1 2; do
  for cfg in "1 8" "2 4"; do
    set -- $cfg
    timeout -k 10 300 python bench.py --steps 8 --warmup 3 --no-coldstart --micro-batch $1 --grad-accum $2 > gpurun_out/ab_mb${1}_r4p_$rep.log 2>&1
    rc=$?; echo "mb=$1 ga=$2 rep=$rep rc=$rc"; [ $rc -ne 0 ] && exit $rc
    echo "mb=$1 ga=$2 rep=$rep $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"max_mem_gb": [0-9.]*' gpurun_out/ab_mb${1}_r4p_$rep.log | tr '\n' ' ')" >> gpurun_out/ab_mb_r4p.txt
  done
done
cat gpurun_out/ab_mb_r4p.txt
