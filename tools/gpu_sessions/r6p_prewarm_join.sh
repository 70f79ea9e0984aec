set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r6p
mkdir -p $O
timeout -k 10 900 python -u bench_apply.py --gpus 1 --runs 3 --steps 1 --warmup 1 \
  --interleave "DSTACK_AMD_PREWARM_JOIN=early,DSTACK_AMD_PREWARM_JOIN=late" > $O/join.json 2> $O/join.err || exit 1
python -c "
import json; d=json.load(open('$O/join.json'))
for k, v in d.items():
    print(k, 'p50 first step', v['first_step_p50_s'], 'p50 submit->step', v['time_to_first_step_p50_s'])
    for s in v['samples']: print('   ', s['time_to_first_step_s'], {a: b for a, b in s['stages_s'].items() if a in ('model_init_s', 'first_step_s', 'imports_s')})
"
