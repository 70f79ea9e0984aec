# fwd attention: 4-stage asm-DMA ring (RING=1) vs 2-stage builtin DMA ring, interleaved same-box runs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2 3; do
  for ring in 1 0; do
    DSTACK_AMD_FA_FWD_RING=$ring timeout -k 10 120 python tools/bench_attn.py > gpurun_out/attn_ring${ring}_$r.json 2>gpurun_out/attn_ring${ring}_$r.err || { echo "bench failed ring=$ring"; tail -5 gpurun_out/attn_ring${ring}_$r.err; exit 1; }
    echo "ring=$ring run=$r $(cat gpurun_out/attn_ring${ring}_$r.json)"
  done
done
