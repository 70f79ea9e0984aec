# first-step split in the applied task with and without the data-pipeline prewarm; then the RCCL
# pre-flight A/B with the probe handed to the runner (--local-probe)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r6k
mkdir -p $O
timeout -k 10 900 python -u bench_apply.py --gpus 1 --runs 3 --steps 1 --warmup 1 --env DSTACK_AMD_FIRST_STEP_SPLIT=1 \
  --interleave "DSTACK_AMD_PREWARM_DATA=0,DSTACK_AMD_PREWARM_DATA=1" > $O/data_prewarm.json 2> $O/data_prewarm.err || exit 1
timeout -k 10 900 python -u bench_apply.py --gpus 1 --runs 3 --steps 1 --warmup 1 --local-probe \
  --interleave "DSTACK_RCCL_PREFLIGHT=0,DSTACK_RCCL_PREFLIGHT=force" > $O/preflight.json 2> $O/preflight.err || exit 1
for f in data_prewarm preflight; do python -c "
import json; d=json.load(open('$O/$f.json'))
for k, v in d.items():
    print(k, 'p50 first step', v['first_step_p50_s'], 'p50 submit->step', v['time_to_first_step_p50_s'])
    for s in v['samples']: print('   ', s['first_step_s'], s['first_step_split'], (s['preflight'] or '')[:90])
"; done
