# Round-3 checkpoint: clipping A/B (loss + step time), GPU suite, smoke, bench, rocprof kernel stats
set -o pipefail
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step noclip timeout -k 10 240 python tools/diag/loss_ab.py --layers 32 --steps 20 > gpurun_out/loss_noclip_r4n.log 2>&1
tail -1 gpurun_out/loss_noclip_r4n.log
step clip timeout -k 10 240 python tools/diag/loss_ab.py --layers 32 --steps 20 --clip 1.0 > gpurun_out/loss_clip_r4n.log 2>&1
tail -1 gpurun_out/loss_clip_r4n.log
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r4n.log 2>&1
step pytest timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r4n.log 2>&1
tail -2 gpurun_out/pytest_r4n.log
exit 0
