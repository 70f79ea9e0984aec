#!/bin/bash
# Same-box A/B of two builds of the package: ./ab_old holds an older dstack_amd (git archive of a
# commit + its own in-tree build) with copies of the entry scripts, which put their own directory
# first on sys.path.  Usage: bash tools/diag/ab_old_new.sh <tag> <gemm SHAPES> <bench steps>
set -o pipefail
TAG=${1:?tag}; SH=${2:-swiglu}; STEPS=${3:-0}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for r in 1 2; do
  timeout -k 10 300 env SHAPES="$SH" python -u ab_old/tools/bench_gemm_nt.py > "$OUT/gemm_old_$r.log" 2>&1 || exit 1
  timeout -k 10 300 env SHAPES="$SH" python -u tools/bench_gemm_nt.py > "$OUT/gemm_new_$r.log" 2>&1 || exit 1
done
if [ "$STEPS" != 0 ]; then
  for r in 1 2; do
    timeout -k 10 600 python -u ab_old/bench.py --gpus 1 --steps "$STEPS" --warmup 2 --no-coldstart > "$OUT/bench_old_$r.log" 2>&1 || exit 1
    timeout -k 10 600 python -u bench.py --gpus 1 --steps "$STEPS" --warmup 2 --no-coldstart > "$OUT/bench_new_$r.log" 2>&1 || exit 1
  done
  for f in "$OUT"/bench_*.log; do echo "$f $(grep -h '"metric"' "$f" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
fi
grep -h "^swiglu\|^km_\|^[a-z_]*_m" "$OUT"/gemm_*.log | cut -c1-220
