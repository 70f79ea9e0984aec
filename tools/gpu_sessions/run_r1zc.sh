set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/diag/overlap_order.py 2>&1 | grep -v amdgpu.ids
