# gradient-precision numbers (printed by the tests) and the concurrent RCCL pre-flight's cost on
# the first optimizer step (bench_apply --interleave, 1 GPU, pre-flight forced vs off)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r6e
timeout -k 10 600 python -u -m pytest -s -x -q --timeout 500 --timeout-method thread -m gpu \
  tests/test_ops_gpu.py::test_gemm_km_grad_accumulation_8_micro_batches_k8192 \
  tests/test_train_gpu.py::test_grad_accum8_bf16_vs_fp32_accumulation > gpurun_out/r6e/precision.log 2>&1 || exit 1
grep -h "rel err\|weight gradients" gpurun_out/r6e/precision.log
timeout -k 10 900 python -u bench_apply.py --gpus 1 --runs 3 --steps 1 --warmup 1 \
  --interleave "DSTACK_RCCL_PREFLIGHT=0,DSTACK_RCCL_PREFLIGHT=force" > gpurun_out/r6e/preflight_ab.json 2> gpurun_out/r6e/preflight_ab.err || exit 1
cut -c1-400 gpurun_out/r6e/preflight_ab.json
