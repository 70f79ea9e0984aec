"""The headline metric end to end on a GPU host: a dstack-amd server (local backend = native
dstack-shim process driver + dstack-runner on this host) receives the Llama-3-8B training task
through the public API (what ``dstack apply`` does), the shim grants a GPU (HIP_VISIBLE_DEVICES),
the runner starts ``bench.py`` as the job, and the tokens/s line is read back from the job's logs.

Prints one JSON line: cold start of THIS task (submit -> running / first log), the job's own bench
result, and the wall time from submit to done.  The parent never touches the GPU (it only runs the
server and reads logs), so the job process is the only GPU user."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from dstack_amd.api import GPU, Resources, Task
    from dstack_amd.server.testing import ServerProcess

    steps = os.environ.get("E2E_STEPS", "5")
    launch = "python"
    if os.environ.get("E2E_TORCHRUN") == "1" or os.environ.get("E2E_LAUNCH") in ("torchrun", "launch"):
        # the examples/llama3-8b-train command: one rank per GPU over the rendezvous env the runner
        # exports, by torchrun or (E2E_LAUNCH=launch, the example's) the torch-free launcher
        prog = "torchrun" if os.environ.get("E2E_LAUNCH", "torchrun") == "torchrun" else "python -m dstack_amd.workloads.launch"
        launch = (f"{prog} --nnodes=$DSTACK_NODES_NUM --node-rank=$DSTACK_NODE_RANK "
                  "--nproc-per-node=$DSTACK_GPUS_PER_NODE --master-addr=$DSTACK_MASTER_NODE_IP "
                  "--master-port=$MASTER_PORT")
    cmd = (f"echo HIP_VISIBLE_DEVICES=$HIP_VISIBLE_DEVICES DSTACK_GPUS_NUM=$DSTACK_GPUS_NUM "
           f"MASTER_ADDR=$DSTACK_MASTER_NODE_IP && cd {ROOT} && "
           f"{launch} bench.py --gpus $DSTACK_GPUS_NUM --steps {steps} --warmup 2 --no-coldstart "
           f"{os.environ.get('E2E_ARGS', '').replace(',', ' ')}")  # E2E_ARGS: comma-separated extra bench args
    # hardware metrics: the server polls the runner's /api/metrics (cgroup + amdsmi) every 2 s here
    # E2E_PROBE=1: the shim hands dstack-probe to the runner, which runs the HIP health probes
    # (HBM, bf16/fp8 MFMA) before the job; the result becomes the instance's health
    # E2E_RCCL_PREFLIGHT=1: the example's RCCL pre-flight, forced for this 1-GPU job (a world of one
    # rank: bootstrap + communicator + an in-place all-reduce, no link bandwidth)
    # E2E_ROCPROF=1: the runner wraps each rank in rocprofv3 (kernel statistics) with the counters
    # of E2E_ROCPROF_COUNTERS, and appends the per-kernel summaries to the job log
    probe = os.environ.get("E2E_PROBE") == "1"
    preflight = os.environ.get("E2E_RCCL_PREFLIGHT") == "1"
    rocprof = os.environ.get("E2E_ROCPROF") == "1"
    srv_env = {"DSTACK_SERVER_METRICS_COLLECT_INTERVAL": "2"}
    if probe or preflight:
        srv_env["DSTACK_LOCAL_GPU_PROBE"] = "1"
    job_env = {"DSTACK_GPU_PROBE": "1"} if probe else {}
    if preflight:
        job_env["DSTACK_RCCL_PREFLIGHT"] = "force"
    if rocprof:
        job_env["DSTACK_ROCPROF"] = "1"
        job_env["DSTACK_ROCPROF_COUNTERS"] = os.environ.get("E2E_ROCPROF_COUNTERS", "SQ_WAVES SQ_INSTS_MFMA")
    with ServerProcess(env=srv_env) as srv:
        client = srv.client()
        conf = Task(name="llama3-8b-e2e", commands=[cmd], resources=Resources(gpu=GPU(count=1)), env=job_env)
        t0 = time.time()
        run = client.runs.submit(conf)
        deadline = t0 + float(os.environ.get("E2E_TIMEOUT", "600"))
        samples = []
        last_print = time.time()
        while time.time() < deadline:
            run.refresh()
            if run.status.is_finished():
                break
            if time.time() - last_print > 20:  # progress for the caller's silence watchdog
                print(f"[e2e] {time.time() - t0:.0f}s status={run.status.value}", flush=True)
                last_print = time.time()
            try:
                jm = client.api.metrics.get_job_metrics("main", run.name, limit=1)
                cur = {m.name: m.values[-1] for m in jm.metrics if m.values}
                if cur:
                    samples.append({k: v for k, v in cur.items() if "gpu" in k or k.startswith("memory")})
            except Exception:  # noqa: BLE001 - metrics appear once the job runs
                pass
            time.sleep(1.0)
        wall = time.time() - t0
        logs = b"".join(run.logs()).decode(errors="replace")
        sub = run.model.jobs[0].job_submissions[-1]
        t = sub.timings or {}
        ts = t.get("submitted", t0)
        bench = None
        for line in logs.splitlines():
            if line.startswith("{") and '"metric"' in line:
                bench = json.loads(line)
        out = {
            "status": sub.status.value,
            "exit_status": sub.exit_status,
            "job_env": [ln for ln in logs.splitlines() if ln.startswith("HIP_VISIBLE_DEVICES")][:1],
            "submit_to_running_s": (t["running"] - ts) if "running" in t else None,
            "submit_to_first_log_s": (t["first_log"] - ts) if "first_log" in t else None,
            "submit_to_done_s": wall,
            "job_bench": bench,
            "hw_metrics_samples": len(samples),
            "hw_metrics_peak": {k: max(x.get(k, 0) for x in samples) for k in (samples[-1] if samples else {})},
        }
        if preflight:
            out["rccl_preflight_log"] = [ln for ln in logs.splitlines() if "RCCL pre-flight" in ln][:1]
        if rocprof:
            lines = logs.splitlines()
            i = next((k for k, ln in enumerate(lines) if "[dstack] rocprofv3" in ln or "DSTACK_ROCPROF" in ln), None)
            out["rocprof_log"] = lines[i:i + 40] if i is not None else []
        if probe or preflight:
            insts = client.api.instances.list(["main"])
            out["instance_health"] = [i.health for i in insts]
            out["probe_log"] = [ln for ln in logs.splitlines() if "GPU health probe" in ln][:1]
        if bench is None:
            out["log_tail"] = logs[-3000:]
            out["server_log_tail"] = srv.log()[-3000:]
        print(json.dumps(out), flush=True)
        return 0 if bench is not None else 1


if __name__ == "__main__":
    sys.exit(main())
