# 70B batch-1 decode at 32k context: kernel timeline of the decode steps (where the 35 ms/token goes)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_r2p
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2p -o run -- python3 bench_serve.py --model llama-3-70b --latency --input-len 32000 --output-len 64 --repeats 1 > gpurun_out/prof_serve_r2p.log 2>&1; echo "prof rc=$?"
tail -1 gpurun_out/prof_serve_r2p.log | cut -c1-500
