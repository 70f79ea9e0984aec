# Grad-norm trace without / with global clipping at 1.0, lr 3e-4 / warmup 100, 20 steps each
# (the unclipped run keeps AdamW inside backward; the clipped one runs it in step())
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python tools/diag/loss_ab.py --layers 32 --steps 20 > gpurun_out/loss_noclip_r4m.log 2>&1
rc=$?; echo "noclip rc=$rc"; tail -1 gpurun_out/loss_noclip_r4m.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python tools/diag/loss_ab.py --layers 32 --steps 20 --clip 1.0 > gpurun_out/loss_clip_r4m.log 2>&1
rc=$?; echo "clip rc=$rc"; tail -1 gpurun_out/loss_clip_r4m.log; exit $rc
