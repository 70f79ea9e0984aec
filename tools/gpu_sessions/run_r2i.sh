# A/B: grid cap of the side-stream AdamW (persistent grid-stride workgroups) 0 = full grid
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
  for b in 0 512 1024 2048 4096; do
    DSTACK_AMD_ADAMW_SIDE_BLOCKS=$b timeout -k 10 300 python -u bench.py --no-coldstart --steps 6 > gpurun_out/ab_sideb${b}_$i.log 2>&1 || { echo "bench b=$b failed"; tail -20 gpurun_out/ab_sideb${b}_$i.log; exit 1; }
    echo "side_blocks=$b run=$i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_sideb${b}_$i.log | tail -1)"
  done
done
