set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r6b
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -v --timeout 500 --timeout-method thread -k "variants_agree" > gpurun_out/r6b/test.log 2>&1; rc=$?; tail -5 gpurun_out/r6b/test.log; [ $rc -eq 0 ] || exit $rc
ARMS="- DSTACK_AMD_FA_DKDV_DEC=1 DSTACK_AMD_FA_DKDV_DEC=1,DSTACK_AMD_FA_DKDV_STAG=12 DSTACK_AMD_FA_DKDV_DEC=1,DSTACK_AMD_FA_DKDV_STAG=24 DSTACK_AMD_FA_DKDV_DEC=1,DSTACK_AMD_FA_DKDV_STAG=40" ROUNDS=2 bash tools/diag/fa_env_ab.sh > gpurun_out/r6b/ab.txt 2>&1 || exit 1
cat gpurun_out/r6b/ab.txt
for arm in "" "DSTACK_AMD_FA_DKDV_DEC=1" "DSTACK_AMD_FA_DKDV_DEC=1 DSTACK_AMD_FA_DKDV_STAG=24"; do
  echo "== trace $arm" >> gpurun_out/r6b/trace.txt
  env $arm timeout -k 10 120 python -u tools/diag/fa_dkdv_phases.py >> gpurun_out/r6b/trace.txt 2>&1 || exit 1
done
cat gpurun_out/r6b/trace.txt
