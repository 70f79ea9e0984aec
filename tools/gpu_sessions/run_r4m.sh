# Grad-norm trace without / with global clipping at 1.0 (AdamW after backward), lr 3e-4 / warmup 100
set -o pipefail
mkdir -p gpurun_out
DSTACK_AMD_OPT_OVERLAP=0 timeout -k 10 240 python tools/diag/loss_ab.py --layers 32 --steps 20 > gpurun_out/loss_noclip_r4m.log 2>&1
rc=$?; echo "noclip rc=$rc"; tail -1 gpurun_out/loss_noclip_r4m.log; [ $rc -ne 0 ] && exit $rc
DSTACK_AMD_OPT_OVERLAP=0 timeout -k 10 240 python tools/diag/loss_ab.py --layers 32 --steps 20 --clip 1.0 > gpurun_out/loss_clip_r4m.log 2>&1
rc=$?; echo "clip rc=$rc"; tail -1 gpurun_out/loss_clip_r4m.log; exit $rc
