# A/B of the forward's K/V DMA form (DSTACK_AMD_FA_FWD_BUF=0|1), interleaved runs of tools/bench_attn.py
set -e
for i in 1 2 3; do
  for v in 0 1; do
    echo "fwd_buf=$v run=$i $(DSTACK_AMD_FA_FWD_BUF=$v timeout -k 10 120 python -u tools/bench_attn.py 2>&1 | grep fwd_ms)"
  done
done
