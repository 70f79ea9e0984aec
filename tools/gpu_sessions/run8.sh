# dkdv variants (64- vs 128-row q stages): numerics + attention timing
set -o pipefail
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest timeout -k 10 600 python -m pytest tests/test_ops_gpu.py -m gpu -x -q -k "flash or attn or llama" > gpurun_out/pytest8.log 2>&1
step pytest128 env DSTACK_AMD_FA_DKDV_QT=128 timeout -k 10 600 python -m pytest tests/test_ops_gpu.py -m gpu -x -q -k "flash or attn or llama" > gpurun_out/pytest8b.log 2>&1
step attn64 timeout -k 10 300 python tools/bench_attn.py > gpurun_out/attn8.json 2> gpurun_out/attn8.err
step attn128 env DSTACK_AMD_FA_DKDV_QT=128 timeout -k 10 300 python tools/bench_attn.py > gpurun_out/attn8b.json 2> gpurun_out/attn8b.err
cat gpurun_out/attn8.json gpurun_out/attn8b.json
