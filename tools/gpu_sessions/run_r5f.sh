# dS^T spill with non-temporal stores in dK/dV vs recompute:
# fp32-reference tests under ds), interleaved timing A/B, rocprofv3 kernel tables of both variants
set -o pipefail
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 300 --timeout-method thread -k "flash" > gpurun_out/pytest_r5f.log 2>&1
tail -1 gpurun_out/pytest_r5f.log
export DSTACK_AMD_FA_DQ=ds
step pytest_ds timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread -k "flash" > gpurun_out/pytest_ds_r5f.log 2>&1
tail -1 gpurun_out/pytest_ds_r5f.log
unset DSTACK_AMD_FA_DQ
: > gpurun_out/fa_dqds_ab_r5f.txt
for i in 1 2 3; do
  for v in recompute ds; do
    r=$(DSTACK_AMD_FA_DQ=$v timeout -k 10 200 python tools/bench_attn.py) || exit 1
    echo "dq=$v rep=$i $r" >> gpurun_out/fa_dqds_ab_r5f.txt
  done
done
cut -c1-200 gpurun_out/fa_dqds_ab_r5f.txt
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in recompute ds; do
  export DSTACK_AMD_FA_DQ=$v
  step prof_$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${v}_r5f -o run -- python3 $R/tools/bench_attn.py > $R/gpurun_out/prof_${v}_r5f.log 2>&1
done
exit 0
