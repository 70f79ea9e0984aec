# batch-1 decode with fp8 weights + fp8 KV: GEMV microbench (bf16 vs fp8) and a kernel profile of single requests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_r3b
timeout -k 10 300 python -u tools/bench_gemv.py > gpurun_out/bench_gemv_r3b.log 2>&1 || { echo "gemv bench failed"; tail -20 gpurun_out/bench_gemv_r3b.log; exit 1; }
grep " 1 {" gpurun_out/bench_gemv_r3b.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3b -o run -- python3 bench_serve.py --model llama-3-70b --quantization fp8 --kv-cache-dtype fp8 --latency --input-len 4096 --output-len 64 --repeats 1 > gpurun_out/prof_serve_r3b.log 2>&1; echo "prof rc=$?"
tail -1 gpurun_out/prof_serve_r3b.log | cut -c1-400
python3 tools/step_breakdown.py gpurun_out/prof_r3b/run_kernel_trace.csv 30 > gpurun_out/decode_step_breakdown_70b_fp8_b1_r3b.txt 2>&1; head -16 gpurun_out/decode_step_breakdown_70b_fp8_b1_r3b.txt
