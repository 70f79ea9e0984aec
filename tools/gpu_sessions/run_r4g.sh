#!/bin/bash
# dK/dV 64-keys-per-wave variants: correctness at S up to 8192, then timing A/B (interleaved)
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for v in 64kv 64k; do
  DSTACK_AMD_FA_DKDV=$v timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 240 \
    --timeout-method thread -k "flash_attention and not variants" > gpurun_out/fa_dkdv_${v}_tests_r4g.log 2>&1 || exit $?
done
for rep in 1 2 3; do
  for v in default 64kv 64k; do
    if [ $v = default ]; then unset DSTACK_AMD_FA_DKDV; else export DSTACK_AMD_FA_DKDV=$v; fi
    echo "== $v rep $rep" >> gpurun_out/fa_dkdv_ab_r4g.txt
    timeout -k 10 120 python -u tools/bench_attn.py >> gpurun_out/fa_dkdv_ab_r4g.txt 2>&1 || exit $?
  done
done
unset DSTACK_AMD_FA_DKDV
