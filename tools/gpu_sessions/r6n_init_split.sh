set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r6n
for i in 1 2 3; do
  timeout -k 10 120 python -u tools/diag/init_split.py >> gpurun_out/r6n/init_split.txt 2>&1 || exit 1
  sleep 5
done
cat gpurun_out/r6n/init_split.txt | grep -v amdgpu.ids
