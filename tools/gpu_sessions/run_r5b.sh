# Fresh-container rebuild at HEAD + the recompute-free dQ pass (DSTACK_AMD_FA_DQ=ds): smoke, full
# GPU suite (variants test covers ds vs default), the S=4096/8192 fp32-reference tests under ds,
# then interleaved timing A/B at the training shape and a rocprofv3 kernel table of each variant
set -o pipefail
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r5b.log 2>&1
step pytest timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r5b.log 2>&1
tail -2 gpurun_out/pytest_r5b.log
export DSTACK_AMD_FA_DQ=ds
step pytest_ds timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread -k "long_seq or flash" > gpurun_out/pytest_ds_r5b.log 2>&1
tail -1 gpurun_out/pytest_ds_r5b.log
unset DSTACK_AMD_FA_DQ
: > gpurun_out/fa_dqds_ab_r5b.txt
for i in 1 2 3; do
  for v in recompute ds; do
    r=$(DSTACK_AMD_FA_DQ=$v timeout -k 10 200 python tools/bench_attn.py) || exit 1
    echo "dq=$v rep=$i $r" >> gpurun_out/fa_dqds_ab_r5b.txt
  done
done
cut -c1-220 gpurun_out/fa_dqds_ab_r5b.txt
cd /tmp && export TMPDIR=/tmp
export DSTACK_AMD_FA_DQ=ds
step prof_ds timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_ds_r5b -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_attn.py > $GRAFT_REPO_ROOT/gpurun_out/prof_ds_r5b.log 2>&1
exit 0
