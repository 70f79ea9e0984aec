#!/bin/bash
# One parameterised GPU session (replaces the per-round one-off scripts that lived in
# tools/gpu_sessions/, see that directory's README): every step runs under its own time limit, the
# steps are chained so that the first failure (or fault, abort, time limit) ends the session, and
# everything lands in gpurun_out/<tag>/.
#
#   bash tools/gpu_session.sh <tag> <step> [<step> ...]
#
# steps:
#   test[=<pytest -k expr>]     pytest -m gpu (optionally a -k selection)
#   smoke                       __graft_entry__.smoke()
#   bench[=<steps>]             python bench.py --steps N --warmup 2 (1 GPU)
#   ab=<steps>:<ENV=a>,<ENV=b>  interleaved same-box A/B of bench.py: a, b, a, b (one env each)
#   prof[=<steps>]              rocprofv3 --kernel-trace --stats over bench.py -> kernel_stats.csv
#   pmc=<c1,c2,...>[@<cmd>]     one rocprofv3 --pmc pass (default command: tools/bench_attn.py)
#   gemm[=<SHAPES>]             tools/bench_gemm_nt.py (in-tree NT GEMM vs hipBLASLt)
#   attn                        tools/bench_attn.py
#   tool=<script.py>            any other measurement script (python -u <script.py>)
#   e2e[=<env assignments>]     tools/e2e_gpu_apply.py (the task through the server, local backend)
#   serve=<bench_serve.py args> bench_serve.py
set -o pipefail
TAG=${1:?usage: gpu_session.sh <tag> <step>...}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1

run() {  # run <name> <seconds> <cmd...>: one step, its own limit, log under $OUT
  local name=$1 secs=$2
  shift 2
  echo "[session] $name: $*" | tee -a "$OUT/session.log"
  local t0=$(date +%s)
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[session] $name: exit $rc after $(( $(date +%s) - t0 )) s" | tee -a "$OUT/session.log"
  tail -n 25 "$OUT/$name.log"
  return $rc
}

for step in "$@"; do
  key=${step%%=*}
  val=""
  [[ "$step" == *=* ]] && val=${step#*=}
  case "$key" in
    test)
      if [ -n "$val" ]; then
        run test 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$val" || exit 1
      else
        run test 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
      fi ;;
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    bench) run bench 600 python -u bench.py --gpus 1 --steps "${val:-8}" --warmup 2 --no-coldstart || exit 1 ;;
    ab)
      steps=${val%%:*}
      arms=${val#*:}
      IFS=',' read -r -a envs <<< "$arms"
      for round in 1 2; do
        i=0
        for e in "${envs[@]}"; do
          i=$((i + 1))
          # shellcheck disable=SC2086
          run "ab_${round}_${i}" 600 env $e python -u bench.py --gpus 1 --steps "$steps" --warmup 2 --no-coldstart || exit 1
          grep -h '"metric"' "$OUT/ab_${round}_${i}.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[ab]', '$e', d['value'], d['ms_per_step'])" | tee -a "$OUT/ab.txt"
        done
      done ;;
    prof)
      run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o k -- \
        python3 -u bench.py --gpus 1 --steps "${val:-5}" --warmup 2 --no-coldstart || exit 1
      find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \; ;;
    pmc)
      ctr=${val%%@*}
      cmd="python3 tools/bench_attn.py"
      [[ "$val" == *@* ]] && cmd=${val#*@}
      # shellcheck disable=SC2086
      run "pmc_$(echo "$ctr" | tr ',' '_' | cut -c1-40)" 240 rocprofv3 --pmc ${ctr//,/ } --output-format csv \
        -d "$OUT/pmc" -o p -- $cmd || exit 1 ;;
    gemm) SHAPES="$val" run gemm 600 python -u tools/bench_gemm_nt.py || exit 1 ;;
    attn) run attn 600 python -u tools/bench_attn.py || exit 1 ;;
    tool) run "$(basename "$val" .py)" 600 python -u "$val" || exit 1 ;;
    e2e)
      # shellcheck disable=SC2086
      run e2e 900 env $val python -u tools/e2e_gpu_apply.py || exit 1 ;;
    serve)
      # shellcheck disable=SC2086
      run serve 1100 python -u bench_serve.py $val || exit 1 ;;
    *) echo "unknown step '$step'"; exit 2 ;;
  esac
done
echo "[session] $TAG: all steps ok" | tee -a "$OUT/session.log"
