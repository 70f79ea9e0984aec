# 70B decode kernel breakdown (rocprofv3 kernel stats) after the attention pipeline + GEMM tuning
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_serve70_r2d -o run -- python3 bench_serve.py --model llama-3-70b --num-prompts 256 --input-len 1024 --output-len 32 > gpurun_out/prof_serve70_r2d.log 2>&1; echo "prof rc=$?"
tail -1 gpurun_out/prof_serve70_r2d.log | cut -c1-600
