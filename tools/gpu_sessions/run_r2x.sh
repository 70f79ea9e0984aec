# kernel trace of the 70B fp8 serving run (decode step breakdown)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_r2x
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2x -o run -- python3 bench_serve.py --model llama-3-70b --quantization fp8 --num-prompts 256 --input-len 1024 --output-len 64 > gpurun_out/prof_serve_r2x.log 2>&1; echo "prof rc=$?"
python3 tools/step_breakdown.py gpurun_out/prof_r2x/run_kernel_trace.csv 20 > gpurun_out/decode_step_breakdown_70b_fp8_r2x.txt 2>&1; cat gpurun_out/decode_step_breakdown_70b_fp8_r2x.txt | head -40
