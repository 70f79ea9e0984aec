# Interleaved same-box A/B of FA environment switches over tools/bench_attn.py:
#   ARMS="ENV=a ENV=b,ENV2=c ..." (comma-separated assignments per arm, "-" = no extra env), ROUNDS (default 3)
set -e
for i in $(seq 1 "${ROUNDS:-3}"); do
  for arm in ${ARMS:?}; do
    if [ "$arm" = "-" ]; then
      r=$(timeout -k 10 120 python -u tools/bench_attn.py 2>&1 | grep fwd_ms)
    else
      # shellcheck disable=SC2086
      r=$(env ${arm//,/ } timeout -k 10 120 python -u tools/bench_attn.py 2>&1 | grep fwd_ms)
    fi
    echo "$arm run=$i $r"
  done
done
