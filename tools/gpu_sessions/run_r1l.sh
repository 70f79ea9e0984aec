# same-box A/B: AdamW side-stream grid cap (optimizer-in-backward) vs full grid vs no overlap
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "adamw or optimizer" > gpurun_out/gpu_tests_r1l.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests_r1l.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r1l.log
run() { # tag env...
  tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-coldstart > gpurun_out/ab_r1l_$tag.log 2>&1 || { echo "bench $tag failed"; tail -20 gpurun_out/ab_r1l_$tag.log; exit 1; }
  echo "$tag $(tail -1 gpurun_out/ab_r1l_$tag.log | grep -o '"ms_per_step": [0-9.]*')"
}
run full DSTACK_AMD_ADAMW_SIDE_BLOCKS=0
run b64 DSTACK_AMD_ADAMW_SIDE_BLOCKS=64
run b32 DSTACK_AMD_ADAMW_SIDE_BLOCKS=32
run b16 DSTACK_AMD_ADAMW_SIDE_BLOCKS=16
run nooverlap DSTACK_AMD_OPT_OVERLAP=0
run b32_2 DSTACK_AMD_ADAMW_SIDE_BLOCKS=32
run full_2 DSTACK_AMD_ADAMW_SIDE_BLOCKS=0
