# A/B: shipped TunableOp GEMM solutions vs hipBLASLt's own heuristics, in the real step, interleaved
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_gemm_tuning_r4q.txt
for rep in 1 2; do
  for mode in use off; do
    DSTACK_AMD_GEMM_TUNING=$mode timeout -k 10 300 python bench.py --steps 8 --warmup 3 --no-coldstart > gpurun_out/ab_gemm_${mode}_r4q_$rep.log 2>&1
    rc=$?; echo "mode=$mode rep=$rep rc=$rc"; [ $rc -ne 0 ] && exit $rc
    echo "gemm_tuning=$mode rep=$rep $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/ab_gemm_${mode}_r4q_$rep.log | tr '\n' ' ')" >> gpurun_out/ab_gemm_tuning_r4q.txt
  done
done
cat gpurun_out/ab_gemm_tuning_r4q.txt
