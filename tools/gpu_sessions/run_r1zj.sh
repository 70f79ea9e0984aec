# checkpoint save/resume on the GPU: pytest + the workload CLI run twice (second run resumes)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_checkpoint.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/ckpt_tests_r1zj.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ckpt_tests_r1zj.log; exit 1; }
tail -1 gpurun_out/ckpt_tests_r1zj.log
rm -rf /tmp/ck_r1zj
timeout -k 10 300 python -u -m dstack_amd.workloads.train_llama --model llama-tiny --seq-len 256 --steps 3 --warmup 0 --checkpoint-dir /tmp/ck_r1zj > gpurun_out/ckpt_run1_r1zj.log 2>&1 || { echo "run1 failed"; tail -10 gpurun_out/ckpt_run1_r1zj.log; exit 1; }
timeout -k 10 300 python -u -m dstack_amd.workloads.train_llama --model llama-tiny --seq-len 256 --steps 3 --warmup 0 --checkpoint-dir /tmp/ck_r1zj > gpurun_out/ckpt_run2_r1zj.log 2>&1 || { echo "run2 failed"; tail -10 gpurun_out/ckpt_run2_r1zj.log; exit 1; }
grep -h "resumed\|step \|loss" gpurun_out/ckpt_run1_r1zj.log gpurun_out/ckpt_run2_r1zj.log | cut -c1-160
cat /tmp/ck_r1zj/meta.json
