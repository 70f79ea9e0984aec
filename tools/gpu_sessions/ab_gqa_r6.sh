# same-box A/B: dK/dV summed over the GQA group in one workgroup (DSTACK_AMD_FA_DKDV_GQA=1, bf16
# straight into dqkv, no fp32 partials / reduce kernel) vs the per-query-head default; numerics
# first (kernel-variants test), then 3 interleaved bench_attn runs each and a kernel-stats pass each
set -o pipefail
O=gpurun_out/ab_gqa_r6
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R && timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py -k "attn or flash" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2 3; do
  DSTACK_AMD_FA_DKDV_GQA=0 timeout -k 10 200 python tools/bench_attn.py > $O/base_$i.json 2>>$O/ab.err || exit 1
  DSTACK_AMD_FA_DKDV_GQA=1 timeout -k 10 200 python tools/bench_attn.py > $O/gqa_$i.json 2>>$O/ab.err || exit 1
done
for i in 1 2; do  # in the training step (the driver's bench, shorter)
  DSTACK_AMD_FA_DKDV_GQA=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/step_base_$i.json 2>>$O/ab.err || exit 1
  DSTACK_AMD_FA_DKDV_GQA=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/step_gqa_$i.json 2>>$O/ab.err || exit 1
done
cd /tmp && export TMPDIR=/tmp
(cd $R && DSTACK_AMD_FA_DKDV_GQA=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_base -o k -- python3 tools/bench_attn.py) > $R/$O/prof_base.log 2>&1 || exit 1
(cd $R && DSTACK_AMD_FA_DKDV_GQA=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_gqa -o k -- python3 tools/bench_attn.py) > $R/$O/prof_gqa.log 2>&1 || exit 1
cd $R
for f in $O/*.json; do echo "$f $(cat $f)"; done
for v in base gqa; do echo "== $v"; find $O/prof_$v -name "*kernel_stats.csv" -exec grep -h "fa_" {} \; | cut -d, -f1-4 | cut -c1-160; done
