# forward attention: deferred-max rescale (DSTACK_AMD_FA_RESCALE_THR) and the software-pipelined
# 8-wave forward (DSTACK_AMD_FA_FWD_PIPE): variant equality + fp32-reference tests, then interleaved
# timing at the training shape (S=8192) and a 32k prefill shape
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "flash or attention" > gpurun_out/fa_tests_r2r.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/fa_tests_r2r.log | head -20; exit 1; }
tail -1 gpurun_out/fa_tests_r2r.log
for rep in 1 2 3; do
  for v in "0 0" "0 8" "1 0" "1 8"; do
    set -- $v
    r=$(DSTACK_AMD_FA_FWD_PIPE=$1 DSTACK_AMD_FA_RESCALE_THR=$2 timeout -k 10 120 python -u tools/bench_attn.py) || { echo "bench failed"; exit 1; }
    echo "rep=$rep pipe=$1 thr=$2 $r" | tee -a gpurun_out/fa_ab_r2r.txt
  done
done
for v in "0 0" "0 8" "1 8"; do
  set -- $v
  r=$(S=32768 DSTACK_AMD_FA_FWD_PIPE=$1 DSTACK_AMD_FA_RESCALE_THR=$2 timeout -k 10 180 python -u tools/bench_attn.py) || { echo "bench32k failed"; exit 1; }
  echo "S=32768 pipe=$1 thr=$2 $r" | tee -a gpurun_out/fa_ab_r2r.txt
done
