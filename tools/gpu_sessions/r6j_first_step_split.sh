set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r6j
mkdir -p $O
timeout -k 10 900 python -u bench_apply.py --gpus 1 --runs 2 --steps 1 --warmup 1 --env DSTACK_AMD_FIRST_STEP_SPLIT=1 \
  --interleave "DSTACK_RCCL_PREFLIGHT=0,DSTACK_RCCL_PREFLIGHT=force" > $O/split.json 2> $O/split.err || exit 1
python -c "
import json; d=json.load(open('$O/split.json'))
for k, v in d.items():
    for s in v['samples']: print(k, s['first_step_s'], s['first_step_split'], s['preflight'])
"
