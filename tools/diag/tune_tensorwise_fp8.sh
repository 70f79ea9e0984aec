# TunableOp selections for the fp8 GEMMs with scalar scales (the deferred-scale prefill path,
# serving/model.py RawScaled) and the row-wise qkv prefill GEMM: results merged into a copy of the
# shipped serving CSV under gpurun_out/ (copy it back to dstack_amd/ops/tuned/ after review).
# BUCKETS / PREFILL_M select the row counts.
cp dstack_amd/ops/tuned/gemm_tunableop_serving_gfx950.csv gpurun_out/serving_tuned.csv
export DSTACK_AMD_GEMM_TUNING_FILE=gpurun_out/serving_tuned.csv
timeout -k 10 500 python -u tools/tune_serving_gemms.py --models llama-3-70b,llama-3-8b --dtype fp8 --scaling tensor \
  --weights wgu,wdown,wo --buckets "${BUCKETS:-128,256}" --prefill-m "${PREFILL_M:-}" --mode tune > gpurun_out/tune_tensor.log 2>&1 &&
timeout -k 10 500 python -u tools/tune_serving_gemms.py --models llama-3-70b,llama-3-8b --dtype fp8 --scaling row \
  --weights wqkv --buckets "${BUCKETS:-128,256}" --prefill-m "${PREFILL_M:-}" --mode tune > gpurun_out/tune_row.log 2>&1
