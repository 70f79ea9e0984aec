# HIP vs torch ops path, full Llama-3-8B, synthetic LM stream, lr 3e-4 / warmup 100, 12 steps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python tools/diag/loss_ab.py --layers 32 --steps 12 > gpurun_out/loss_ab_hip_r4l.log 2>&1
rc=$?; echo "hip rc=$rc"; tail -1 gpurun_out/loss_ab_hip_r4l.log; [ $rc -ne 0 ] && exit $rc
DSTACK_AMD_OPS=torch timeout -k 10 400 python tools/diag/loss_ab.py --layers 32 --steps 12 > gpurun_out/loss_ab_torch_r4l.log 2>&1
rc=$?; echo "torch rc=$rc"; tail -1 gpurun_out/loss_ab_torch_r4l.log; exit $rc
