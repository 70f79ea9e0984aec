set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r6q
timeout -k 10 300 python -u tools/diag/cu_hog.py > gpurun_out/r6q/persistent.txt 2>&1 || exit 1
DSTACK_AMD_GEMM_NT_PERSISTENT=0 timeout -k 10 300 python -u tools/diag/cu_hog.py > gpurun_out/r6q/nonpersistent.txt 2>&1 || exit 1
grep -v "^{\|amdgpu.ids" gpurun_out/r6q/persistent.txt; echo "-- one workgroup per tile:"; grep -v "^{\|amdgpu.ids" gpurun_out/r6q/nonpersistent.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread -m gpu tests/test_ops_gpu.py -k "long_k or k8192" > gpurun_out/r6q/gemm_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r6q/gemm_tests.log; exit $rc
