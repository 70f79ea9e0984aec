# same-box full-bench A/B of the attention wave-count switches (ms/step, 2 rounds interleaved)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-coldstart > gpurun_out/ab_r1za_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/ab_r1za_$tag.log; exit 1; }
  echo "$tag $(tail -1 gpurun_out/ab_r1za_$tag.log | grep -o '"ms_per_step": [0-9.]*')"; }
for r in 1 2; do
  run fwd8_dq8_$r DSTACK_AMD_FA_FWD_WAVES=8
  run fwd4_dq8_$r DSTACK_AMD_FA_FWD_WAVES=4
  run fwd4_dq4_$r DSTACK_AMD_FA_FWD_WAVES=4 DSTACK_AMD_FA_DQ_WAVES=4
done
