# Power / GFX clock during the bench step (is the step power-capped?) + docker availability on the box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/diag/power_trace.py --steps 6 > gpurun_out/power_trace_r4s.log 2>&1
rc=$?; echo "power rc=$rc"; tail -1 gpurun_out/power_trace_r4s.log
(command -v docker && docker info --format '{{.ServerVersion}}') > gpurun_out/docker_r4s.txt 2>&1; echo "docker: $(head -c 300 gpurun_out/docker_r4s.txt)"
exit $rc
