# LR warmup sweep on the synthetic LM stream (Llama-3-8B, S=8192, grad-accum 8): 30 steps each
set -o pipefail
mkdir -p gpurun_out
for cfg in "3e-4 100" "3e-4 300" "1e-4 100"; do
  set -- $cfg
  timeout -k 10 300 python -m dstack_amd.workloads.train_llama --steps 25 --warmup 5 --grad-accum 8 \
      --lr $1 --lr-warmup $2 > gpurun_out/lr_sweep_${1}_${2}_r4k.log 2>&1
  rc=$?; echo "lr=$1 warmup=$2 rc=$rc"; [ $rc -ne 0 ] && exit $rc
  grep -o '"losses": \[[^]]*\]' gpurun_out/lr_sweep_${1}_${2}_r4k.log
done
exit 0
