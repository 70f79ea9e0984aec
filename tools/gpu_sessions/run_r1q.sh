set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
true
true
for v in a b; do
timeout -k 10 200 python -u tools/bench_ops.py > gpurun_out/ops_cap_default_$v.json 2>&1 || { tail -5 gpurun_out/ops_cap_default_$v.json; exit 1; }
DSTACK_AMD_GRID_CAP=0 timeout -k 10 200 python -u tools/bench_ops.py > gpurun_out/ops_cap0_$v.json 2>&1 || { tail -5 gpurun_out/ops_cap0_$v.json; exit 1; }
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/ops_cap*.json')):
    txt=open(f).read(); i=txt.index('{'); d=json.loads(txt[i:txt.rindex('}')+1])
    print(f, {k: round(v,3) for k,v in d.items() if k.endswith('_ms') or k=='adamw_TBps'})
PY
for v in a b; do
timeout -k 10 300 python -u bench.py --no-coldstart > gpurun_out/bench_cap_default_$v.log 2>&1 || exit 1
DSTACK_AMD_GRID_CAP=0 timeout -k 10 300 python -u bench.py --no-coldstart > gpurun_out/bench_cap0_$v.log 2>&1 || exit 1
echo "default $(tail -1 gpurun_out/bench_cap_default_$v.log | grep -o '"ms_per_step": [0-9.]*')  cap0 $(tail -1 gpurun_out/bench_cap0_$v.log | grep -o '"ms_per_step": [0-9.]*')"
done
