# same-box A/B of the dK/dV kernels: 4-wave (default) vs 8-wave K/V-resident (DSTACK_AMD_FA_DKDV=8w)
set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  timeout -k 10 200 python tools/bench_attn.py > gpurun_out/ab4_$i.json 2>>gpurun_out/ab.err || exit 1
  DSTACK_AMD_FA_DKDV=8w timeout -k 10 200 python tools/bench_attn.py > gpurun_out/ab8_$i.json 2>>gpurun_out/ab.err || exit 1
done
for f in gpurun_out/ab4_*.json gpurun_out/ab8_*.json; do echo "$f $(cat $f)"; done
