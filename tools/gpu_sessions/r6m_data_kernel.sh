# the synthetic stream's HIP kernel: bit-identical to the CPU definition; the applied task's first
# step split and stages with it (3 fresh-instance runs)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r6m
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_ops_gpu.py -k synthetic_tokens > $O/test.log 2>&1; rc=$?; tail -4 $O/test.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u bench_apply.py --gpus 1 --runs 3 --steps 1 --warmup 1 --env DSTACK_AMD_FIRST_STEP_SPLIT=1 \
  --interleave "DSTACK_AMD_FIRST_STEP_SPLIT=1" > $O/split.json 2> $O/split.err || exit 1
python -c "
import json; d=json.load(open('$O/split.json'))
for k, v in d.items():
    print(k, 'p50 first step', v['first_step_p50_s'], 'p50 submit->step', v['time_to_first_step_p50_s'])
    for s in v['samples']: print('   ', s['first_step_split'], s['stages_s'])
"
