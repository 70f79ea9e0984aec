# same-box A/B: optimizer-in-backward on/off (whole training step)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for ov in 0 1; do
    DSTACK_AMD_OPT_OVERLAP=$ov timeout -k 10 300 python bench.py --no-coldstart --steps 5 --warmup 2 > gpurun_out/ab_opt_${ov}_$i.log 2>&1 || exit 1
    echo "ov=$ov $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_opt_${ov}_$i.log)"
  done
done
