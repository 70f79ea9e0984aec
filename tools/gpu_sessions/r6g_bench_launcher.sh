# the driver's N>1 form at N=1: torch.distributed.run ... bench.py (cold start on rank 0 after the
# timed steps, once the trainer is closed and the caches emptied)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r6g
mkdir -p $O
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29551 \
  bench.py --gpus 1 --steps 5 --warmup 2 > $O/bench_launcher.log 2>&1 || exit 1
grep '^{\|warning' $O/bench_launcher.log | cut -c1-300
