# A/B of the backward's S/dP read pipelines: DSTACK_AMD_FA_DKDV_PF (dK/dV pass) and DSTACK_AMD_FA_DQ_PF
# (dQ pass), interleaved runs of tools/bench_attn.py; VARIANTS = "dkdvpf:dqpf ..."
set -e
for i in 1 2 3; do
  for v in ${VARIANTS:-0:0 2:0 2:1 2:2}; do
    a=${v%%:*}; b=${v##*:}
    echo "dkdv_pf=$a dq_pf=$b run=$i $(DSTACK_AMD_FA_DKDV_PF=$a DSTACK_AMD_FA_DQ_PF=$b timeout -k 10 120 python -u tools/bench_attn.py 2>&1 | grep fwd_ms)"
  done
done
