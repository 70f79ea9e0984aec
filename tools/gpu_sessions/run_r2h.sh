# A/B: compute on a high-priority stream (AdamW side stream at normal priority) vs one priority
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
  for p in 0 1; do
    DSTACK_AMD_MAIN_PRIO=$p timeout -k 10 300 python -u bench.py --no-coldstart --steps 6 > gpurun_out/ab_prio${p}_$i.log 2>&1 || { echo "bench prio=$p failed"; tail -20 gpurun_out/ab_prio${p}_$i.log; exit 1; }
    echo "prio=$p run=$i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_prio${p}_$i.log | tail -1)"
  done
done
bash tools/prof_tag.sh r2h
