# serving: single 32k-token prompt latency (70B, 1 GPU; the reference's large-prompt figure is 405B FP8 on
# 8xMI300X) and a kernel profile of the 70B throughput run's decode steps
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u bench_serve.py --model llama-3-70b --latency --input-len 32000 --output-len 128 --repeats 2 > gpurun_out/serve_70b_latency32k_r2n.log 2>&1 || { echo "latency bench failed"; tail -30 gpurun_out/serve_70b_latency32k_r2n.log; exit 1; }
tail -1 gpurun_out/serve_70b_latency32k_r2n.log | cut -c1-900
mkdir -p gpurun_out/prof_r2n
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2n -o run -- python3 bench_serve.py --model llama-3-70b --num-prompts 256 --input-len 1024 --output-len 64 > gpurun_out/prof_serve_r2n.log 2>&1; echo "prof rc=$?"
tail -1 gpurun_out/prof_serve_r2n.log | cut -c1-600
