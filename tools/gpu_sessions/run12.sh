# GEMM: plain vs L2 warm-up prefetch distance
set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
TAGS=""
run() { local tag=$1; shift; TAGS="$TAGS $tag"; env "$@" timeout -k 10 300 python tools/bench_gemm.py > gpurun_out/gemm12_$tag.log 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/gemm12_$tag.log; exit 1; }; }
run plain DSTACK_AMD_GEMM_TN=plain
run pf1 DSTACK_AMD_GEMM_TN=pf1
run pf2 DSTACK_AMD_GEMM_TN=pf2
run pf3 DSTACK_AMD_GEMM_TN=pf3
for t in $TAGS; do echo "== $t"; grep -v "^{" gpurun_out/gemm12_$t.log | grep -v amdgpu.ids | python -c "
import sys, json
for l in sys.stdin:
    n, j = l.split(' ', 1); j = json.loads(j)
    print(n, round(j['hip_tflops']), round(j['lib_tflops']), round(j['hip_acc_ms'], 3), '%.4f %.4f' % (j['rel_err'], j['rel_err_acc']))
"; done
