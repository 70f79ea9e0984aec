set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r6i
mkdir -p $O
for arm in "--prewarm" "--prewarm --warm-data"; do
  echo "== $arm" >> $O/first_step.txt
  timeout -k 10 300 python -u tools/diag/first_step.py $arm >> $O/first_step.txt 2>&1 || exit 1
  sleep 20
done
grep "==\|step 0\|step 1\|setup\|throwaway" $O/first_step.txt | cut -c1-160
