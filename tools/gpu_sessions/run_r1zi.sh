# same-box A/B: HEAD vs e7ab7e5 (the 21.30k tok/s build, checked out under ab_u/), interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-coldstart > gpurun_out/ab_head_$r.log 2>&1 || { echo "head bench failed"; tail -5 gpurun_out/ab_head_$r.log; exit 1; }
  echo "head run=$r $(tail -1 gpurun_out/ab_head_$r.log | cut -c150-260)"
  (cd ab_u && timeout -k 10 300 python -u bench.py --no-coldstart > ../gpurun_out/ab_old_$r.log 2>&1) || { echo "old bench failed"; tail -5 gpurun_out/ab_old_$r.log; exit 1; }
  echo "old  run=$r $(tail -1 gpurun_out/ab_old_$r.log | cut -c150-260)"
done
