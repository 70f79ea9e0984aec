# paged decode attention in isolation: layout x split plan
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_paged_decode.py > gpurun_out/bench_paged_decode_r2e.jsonl 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_paged_decode_r2e.jsonl; exit 1; }
grep -c TBps gpurun_out/bench_paged_decode_r2e.jsonl
