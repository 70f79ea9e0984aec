# start-up after dropping the TunableOp / device-properties calls and the fp32->bf16 model copy
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r6o
mkdir -p $O
timeout -k 10 900 python -u bench_apply.py --gpus 1 --runs 3 --steps 1 --warmup 1 \
  --interleave "DSTACK_AMD_FIRST_STEP_SPLIT=0" > $O/startup.json 2> $O/startup.err || exit 1
python -c "
import json; d=json.load(open('$O/startup.json'))
for k, v in d.items():
    print(k, 'p50 first step', v['first_step_p50_s'], 'p50 submit->step', v['time_to_first_step_p50_s'])
    for s in v['samples']: print('   ', s['time_to_first_step_s'], s['stages_s'])
"
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_train_gpu.py -k loss_falls > $O/train_test.log 2>&1; rc=$?; tail -3 $O/train_test.log; exit $rc
