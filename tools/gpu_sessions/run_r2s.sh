# SIMD-balanced wave slots in the causal 8-wave attention kernels (DSTACK_AMD_FA_SIMD_BAL) and the
# unscheduled pipelined forward (DSTACK_AMD_FA_FWD_PIPE=2): variant tests, interleaved timing
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "flash or attention" > gpurun_out/fa_tests_r2s.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/fa_tests_r2s.log | head -20; exit 1; }
tail -1 gpurun_out/fa_tests_r2s.log
for rep in 1 2 3; do
  for v in "0 0" "0 1" "2 1"; do
    set -- $v
    r=$(DSTACK_AMD_FA_FWD_PIPE=$1 DSTACK_AMD_FA_SIMD_BAL=$2 timeout -k 10 120 python -u tools/bench_attn.py) || { echo "bench failed"; exit 1; }
    echo "rep=$rep pipe=$1 bal=$2 $r" | tee -a gpurun_out/fa_ab_r2s.txt
  done
done
