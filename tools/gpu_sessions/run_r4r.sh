# A/B: s_setprio in the flash-attention forward (DSTACK_AMD_FA_PRIO 0 / 1 = MFMA phases high /
# 2 = softmax phase high), 3 interleaved runs each; bench_attn also checks accuracy vs fp32 SDPA
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/fa_prio_ab_r4r.txt
for rep in 1 2 3; do
  for prio in 0 1 2; do
    DSTACK_AMD_FA_PRIO=$prio timeout -k 10 120 python tools/bench_attn.py > gpurun_out/fa_prio_${prio}_r4r_$rep.json 2> gpurun_out/fa_prio_${prio}_r4r_$rep.err
    rc=$?; echo "prio=$prio rep=$rep rc=$rc"; [ $rc -ne 0 ] && exit $rc
    echo "prio=$prio rep=$rep $(tr -d '\n' < gpurun_out/fa_prio_${prio}_r4r_$rep.json)" >> gpurun_out/fa_prio_ab_r4r.txt
  done
done
cut -c1-200 gpurun_out/fa_prio_ab_r4r.txt
