# the driver's bench forms with the cold start: no launcher (cold start before the ranks) and under
# torch.distributed.run (cold start on rank 0 after the timed steps); plus the first-step split
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r6f
mkdir -p $O
timeout -k 10 300 python -u tools/diag/first_step.py > $O/first_step.log 2>&1 || exit 1
grep "step\|setup" $O/first_step.log
timeout -k 10 900 python -u bench.py --steps 5 --warmup 2 > $O/bench_nolauncher.log 2>&1 || exit 1
grep '^{' $O/bench_nolauncher.log | cut -c1-300
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29551 \
  bench.py --gpus 1 --steps 5 --warmup 2 > $O/bench_launcher.log 2>&1 || exit 1
grep '^{' $O/bench_launcher.log | cut -c1-300
