set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r6c
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -v --timeout 500 --timeout-method thread -k "variants_agree" > gpurun_out/r6c/test.log 2>&1; rc=$?; tail -3 gpurun_out/r6c/test.log; [ $rc -eq 0 ] || exit $rc
ARMS="- DSTACK_AMD_FA_DKDV_DEC=1 DSTACK_AMD_FA_DKDV_DEC=2 DSTACK_AMD_FA_DKDV_DEC=2,DSTACK_AMD_FA_DKDV_STAG=24" ROUNDS=3 bash tools/diag/fa_env_ab.sh > gpurun_out/r6c/ab.txt 2>&1 || exit 1
cat gpurun_out/r6c/ab.txt | sed 's/"fwd_max_err.*//'
echo "== trace DEC=2" >> gpurun_out/r6c/trace.txt
DSTACK_AMD_FA_DKDV_DEC=2 timeout -k 10 120 python -u tools/diag/fa_dkdv_phases.py >> gpurun_out/r6c/trace.txt 2>&1 || exit 1
cat gpurun_out/r6c/trace.txt
