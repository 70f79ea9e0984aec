# FA: static priority for waves 4-7 (DSTACK_AMD_FA_HALF_PRIO=1) in the 8-wave forward, dK/dV and dQ
# passes vs default -- numerics, then four interleaved timing runs at the training shape
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 300 --timeout-method thread \
  -k "kernel_variants_agree" > gpurun_out/fa_hprio_tests_r4y.log 2>&1
rc=$?; tail -2 gpurun_out/fa_hprio_tests_r4y.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/fa_hprio_ab_r4y.txt
for i in 1 2 3 4; do
  for v in 0 1; do
    r=$(DSTACK_AMD_FA_HALF_PRIO=$v timeout -k 10 200 python tools/bench_attn.py) || exit 1
    echo "half_prio=$v rep=$i $r" >> gpurun_out/fa_hprio_ab_r4y.txt
  done
done
cut -c1-150 gpurun_out/fa_hprio_ab_r4y.txt
