# same-box A/B of flash-attention builds: .ab_old (HEAD kernels) vs the current tree: numerics tests
# of the current tree, 3 interleaved bench_attn runs each, and one rocprofv3 kernel-stats pass each
# (per-kernel split of the backward)
set -o pipefail
O=gpurun_out/ab_r6
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd $R && timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "attn or flash" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2 3; do
  (cd $R/.ab_old && timeout -k 10 200 python tools/bench_attn.py) > $O/old_$i.json 2>>$O/ab.err || exit 1
  (cd $R && timeout -k 10 200 python tools/bench_attn.py) > $O/new_$i.json 2>>$O/ab.err || exit 1
done
cd /tmp && export TMPDIR=/tmp
(cd $R/.ab_old && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof_old -o k -- python3 tools/bench_attn.py) > $R/$O/prof_old.log 2>&1 || exit 1
(cd $R && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof_new -o k -- python3 tools/bench_attn.py) > $R/$O/prof_new.log 2>&1 || exit 1
cd $R
for f in $O/*.json; do echo "$f $(cat $f)"; done
for v in old new; do echo "== $v"; find $O/prof_$v -name "*kernel_stats.csv" -exec grep fa_ {} \; | cut -d, -f1-4; done
