# weight-gradient GEMM kernel: accuracy + timing vs hipBLASLt at the Llama-3-8B shapes, per pipeline variant
set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
for v in plain pipe; do
  DSTACK_AMD_GEMM_TN=$v timeout -k 10 300 python tools/bench_gemm.py > gpurun_out/gemm11_$v.log 2>&1 || { echo "gemm $v failed"; tail -5 gpurun_out/gemm11_$v.log; exit 1; }
done
for v in plain pipe; do echo "== $v"; grep -v "^{" gpurun_out/gemm11_$v.log | grep -v amdgpu.ids | python -c "
import sys, json
for l in sys.stdin:
    n, j = l.split(' ', 1); j = json.loads(j)
    print(n, round(j['hip_tflops']), round(j['lib_tflops']), round(j['hip_acc_ms'], 3), '%.4f' % j['rel_err'])
"; done
