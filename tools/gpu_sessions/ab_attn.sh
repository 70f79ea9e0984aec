# same-box A/B of flash-attention builds: .ab_old (previous kernels) vs the current tree
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for i in 1 2 3; do
  (cd $R/.ab_old && timeout -k 10 200 python tools/bench_attn.py) > gpurun_out/ab_old_$i.json 2>>gpurun_out/ab.err || exit 1
  (cd $R && timeout -k 10 200 python tools/bench_attn.py) > gpurun_out/ab_new_$i.json 2>>gpurun_out/ab.err || exit 1
  (cd $R && DSTACK_AMD_FA_DKDV_QT=128 timeout -k 10 200 python tools/bench_attn.py) > gpurun_out/ab_new128_$i.json 2>>gpurun_out/ab.err || exit 1
done
for f in gpurun_out/ab_*.json; do echo "$f $(cat $f)"; done
