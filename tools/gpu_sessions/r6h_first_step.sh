# first optimizer step vs steady steps, with the GEMM prewarm as run() does, and with the first
# step's activation pool reserved beside model init (DSTACK_AMD_ACT_POOL_GB)
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r6h
mkdir -p $O
for arm in "--prewarm" "--prewarm --pool-gb 40" "--prewarm --pool-gb 100" "--prewarm"; do
  echo "== $arm" >> $O/first_step.txt
  timeout -k 10 300 python -u tools/diag/first_step.py $arm >> $O/first_step.txt 2>&1 || exit 1
done
grep "==\|step 0\|step 1\|setup" $O/first_step.txt | cut -c1-200
