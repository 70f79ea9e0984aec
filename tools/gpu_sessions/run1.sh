set -o pipefail
mkdir -p gpurun_out
(amd-smi static --asic --vram --bus --json > gpurun_out/amdsmi_static.json 2>&1; amd-smi topology --json > gpurun_out/amdsmi_topo.json 2>&1; rocminfo > gpurun_out/rocminfo.txt 2>&1) || true
timeout -k 10 400 python tools/gpu_diag.py > gpurun_out/diag.json 2> gpurun_out/diag.err && \
DSTACK_AMD_OPS=torch timeout -k 10 500 python bench.py --steps 3 --warmup 2 > gpurun_out/bench_torch.log 2>&1
echo EXIT $?
