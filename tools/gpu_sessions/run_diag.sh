set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/diag/step_check.py && DSTACK_AMD_OPT_OVERLAP=0 timeout -k 10 120 python -u tools/diag/step_check.py && MODEL=llama-3-8b SEQ=8192 timeout -k 10 200 python -u tools/diag/step_check.py
