# same-box A/B of the forward's deferred-rescale threshold (P <= 2^thr): default 8 vs 10 and 12
set -o pipefail
O=gpurun_out/ab_rescale_r6f
mkdir -p $O
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  for t in 8 10 12; do
    DSTACK_AMD_FA_RESCALE_THR=$t timeout -k 10 200 python tools/bench_attn.py > $O/thr${t}_$i.json 2>>$O/err.log || exit 1
  done
done
for f in $O/*.json; do echo "$f $(cat $f)"; done
