# Early-training stability at the bench shape (32 layers, 8 x 8192 tokens/step, lr 3e-4, 300-step
# warmup, synthetic-lm stream): default output-head init (std 0.02) vs zero-init vs std 0.02/sqrt(2L)
set -o pipefail
mkdir -p gpurun_out
for v in default 0 0.0025; do
  extra=""; [ "$v" != default ] && extra="--lm-head-std $v"
  timeout -k 10 300 python -u tools/diag/loss_ab.py --layers 32 --steps 25 --lr 3e-4 --lr-warmup 300 $extra \
    > gpurun_out/lmhead_${v}_r4aa.log 2>&1 || { echo "$v rc=$?"; tail -5 gpurun_out/lmhead_${v}_r4aa.log; exit 1; }
  tail -1 gpurun_out/lmhead_${v}_r4aa.log | cut -c1-400
done
