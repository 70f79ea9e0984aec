# FA forward: staggered SIMD partners (DSTACK_AMD_FA_FWD_STAG=1) vs default -- numerics, then
# three interleaved timing runs at the training shape
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 300 --timeout-method thread \
  -k "kernel_variants_agree or flash_attention" > gpurun_out/fa_stag_tests_r4x.log 2>&1
rc=$?; tail -2 gpurun_out/fa_stag_tests_r4x.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/fa_stag_ab_r4x.txt
for i in 1 2 3; do
  for v in 0 1; do
    r=$(DSTACK_AMD_FA_FWD_STAG=$v timeout -k 10 200 python tools/bench_attn.py) || exit 1
    echo "stag=$v rep=$i $r" >> gpurun_out/fa_stag_ab_r4x.txt
  done
done
cat gpurun_out/fa_stag_ab_r4x.txt
