# Per-kernel stats of the 70B fp8+fp8kv serving run with the fp8 scale deferral from 256 rows
# (decode batch included) and from 1024 rows (prefill only)
set -o pipefail
export TMPDIR=/tmp
for r in 256 1024; do
  DSTACK_AMD_FP8_DEFER_ROWS=$r timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/sp$r -o k -- python3 -u bench_serve.py --model llama-3-70b --quantization fp8 \
    --kv-cache-dtype fp8 --output-len 128 > gpurun_out/sp$r.log 2>&1 || exit 1
  find gpurun_out/sp$r -name "*kernel_stats.csv" -exec cp {} gpurun_out/sp${r}_stats.csv \;
  rm -rf gpurun_out/sp$r  # the raw traces exceed what gpurun copies back
done
