# dynamic per-XCD tile queue in the persistent GEMM: correctness, behaviour beside held CUs, step A/B
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r6s
mkdir -p $O
DSTACK_AMD_GEMM_NT_DYNAMIC=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread -m gpu tests/test_ops_gpu.py -k "gemm_nt or gemm_km or mlp" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
DSTACK_AMD_GEMM_NT_DYNAMIC=1 timeout -k 10 300 python -u tools/diag/cu_hog.py > $O/hog_dynamic.txt 2>&1 || exit 1
grep -v "^{\|amdgpu.ids" $O/hog_dynamic.txt
bash tools/gpu_session.sh r6s_ab "ab=6:DSTACK_AMD_GEMM_NT_DYNAMIC=0,DSTACK_AMD_GEMM_NT_DYNAMIC=1" > /dev/null 2>&1 || exit 1
cat gpurun_out/r6s_ab/ab.txt
