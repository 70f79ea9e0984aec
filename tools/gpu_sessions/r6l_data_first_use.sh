set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r6l
timeout -k 10 120 python -u tools/diag/data_first_use.py > gpurun_out/r6l/data_first_use.txt 2>&1 || exit 1
timeout -k 10 120 python -u tools/diag/data_first_use.py >> gpurun_out/r6l/data_first_use.txt 2>&1 || exit 1
cat gpurun_out/r6l/data_first_use.txt
