"""Job cold-start benchmark: the first half of BASELINE's headline metric ("p50 job cold-start (s)").

Starts a real dstack-amd server (local backend: native ``dstack-shim`` process driver +
``dstack-runner``) and ``apply``s tasks through the public API, reading each job's stage
timestamps:

* ``submit_to_running``   : API submit  -> runner started the user command
* ``submit_to_first_log`` : API submit  -> first byte of job output (runner clock)

Two series, reported separately:

* **fresh** (``cold_start_p50_s``): every run lands on a NEW instance with its OWN freshly started
  agent -- the previous run's fleet is deleted, its instance terminated and its shim stopped first
  (local backend in per-instance-agent mode, ``DSTACK_LOCAL_SHIM_PER_INSTANCE=1``), so each run goes
  through offer selection, instance creation, agent start (``dstack-shim --host-info``, process
  start, first healthcheck), GPU grant, runner start and the job's first output.  ``stages_p50_s``
  splits it: offer + instance record, agent start, task/runner start, user command to first log.  With a GPU on the host (``--gpu auto``)
  the task requests ``MI355X:1``, so the xGMI-aware pick, ``HIP_VISIBLE_DEVICES`` and the runner's
  GPU env are in the measured path.
* **warm** (``warm_start_p50_s``): runs that reuse the idle instance of the previous run (the
  reference's pool reuse).

What is NOT in either number (and is in the reference's cloud cold start): VM boot, image pull and
container start -- the local backend runs the job as a process on the server's host.  The number is
the control plane's own latency, not a cloud provisioning time.
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time


def _host_has_gpu() -> bool:
    try:
        from dstack_amd import native_bin

        shim = native_bin.shim_path()
        if not shim:
            return False
        out = subprocess.run([shim, "--list-gpus"], capture_output=True, text=True, timeout=60).stdout
        return bool(json.loads(out.strip().splitlines()[-1]).get("amdsmi"))
    except Exception:  # noqa: BLE001
        return False


def _sample(run, t0):
    sub = run.model.jobs[0].job_submissions[-1]
    t = sub.timings or {}
    base = t.get("submitted", t0)
    agent = {}
    if sub.job_provisioning_data and sub.job_provisioning_data.backend_data:
        try:
            agent = json.loads(sub.job_provisioning_data.backend_data).get("agent") or {}
        except ValueError:
            agent = {}
    return {
        "agent": agent,
        "submit_to_container_running": _d(t, "container_running", base),
        "status": sub.status.value,
        "termination_reason": sub.termination_reason.value if sub.termination_reason else None,
        "message": sub.termination_reason_message,
        "submit_to_provisioned": _d(t, "provisioned", base) or _d(t, "assigned", base),
        "submit_to_running": _d(t, "running", base),
        "submit_to_first_log": _d(t, "first_log", base),
        "client_wall_to_done": round(time.time() - t0, 4),
        "instance": (sub.job_provisioning_data.instance_id if sub.job_provisioning_data else None),
    }


def _retire_instances(client, project="main", timeout=60.0):
    """Delete every fleet (terminating its idle instances) and wait until none is active, so the
    next run has to create a fresh instance."""
    api = client.api
    fleets = [f.name for f in api.fleets.list(project)]
    if fleets:
        api.fleets.delete(project, fleets)
    deadline = time.time() + timeout
    while time.time() < deadline:
        active = [i for i in api.instances.list([project], only_active=True)
                  if i.status.value not in ("terminating", "terminated")]
        if not active:
            return True
        time.sleep(0.05)
    return False


def measure_cold_start(runs: int = 5, warm_runs: int = 4, timeout: float = 120.0, command: str = "echo ready",
                       gpu: str = "auto") -> dict:
    from dstack_amd.api import Resources, Task
    from dstack_amd.server.testing import ServerProcess

    use_gpu = _host_has_gpu() if gpu == "auto" else gpu == "yes"
    fresh, warm, errors = [], [], []
    # one agent per instance: a fresh instance's agent start is inside its job's cold start
    with ServerProcess(env={"DSTACK_LOCAL_SHIM_PER_INSTANCE": "1"}) as srv:
        client = srv.client()
        for i in range(runs + warm_runs):
            is_fresh = i < runs
            if is_fresh and i > 0 and not _retire_instances(client):
                errors.append(f"run {i}: previous instance still active")
            kw = {"resources": Resources(gpu="MI355X:1")} if use_gpu else {}
            conf = Task(commands=[command], name=f"coldstart-{i}", **kw)
            t0 = time.time()
            run = client.runs.submit(conf)
            run.wait(timeout=timeout, poll=0.05)
            s = _sample(run, t0)
            (fresh if is_fresh else warm).append(s)
            if s["submit_to_first_log"] is None:
                errors.append(f"run {i}: {s}")
                print(f"coldstart run {i} failed: {s}", file=sys.stderr)
                print(srv.log()[-4000:], file=sys.stderr)
    ok_f = [s for s in fresh if s["submit_to_first_log"] is not None]
    ok_w = [s for s in warm if s["submit_to_first_log"] is not None]
    med = (lambda xs, k: round(statistics.median([x[k] for x in xs]), 4) if xs else None)
    distinct = len({s["instance"] for s in fresh if s["instance"]})

    def p50(xs):
        xs = [x for x in xs if x is not None]
        return round(statistics.median(xs), 4) if xs else None

    agent_s = [s["agent"].get("agent_start_s") for s in ok_f]
    stages = {
        "offer_and_instance_s": p50([s["submit_to_provisioned"] - s["agent"].get("agent_start_s", 0.0)
                                     for s in ok_f if s["submit_to_provisioned"] is not None]),
        "agent_start_s": p50(agent_s),
        "agent_host_info_s": p50([s["agent"].get("host_info_s") for s in ok_f]),
        "task_and_runner_start_s": p50([s["submit_to_running"] - s["submit_to_provisioned"] for s in ok_f
                                        if s["submit_to_running"] is not None and s["submit_to_provisioned"] is not None]),
        "command_to_first_log_s": p50([s["submit_to_first_log"] - s["submit_to_running"] for s in ok_f
                                       if s["submit_to_running"] is not None]),
    }
    return {
        "cold_start_p50_s": med(ok_f, "submit_to_first_log"),
        "stages_p50_s": stages,
        "fresh_agent_per_instance": all(s["agent"] for s in ok_f) and bool(ok_f),
        "cold_running_p50_s": med(ok_f, "submit_to_running"),
        "warm_start_p50_s": med(ok_w, "submit_to_first_log"),
        "gpu_requested": "MI355X:1" if use_gpu else None,
        "fresh_runs": len(fresh), "fresh_ok": len(ok_f), "fresh_distinct_instances": distinct,
        "warm_runs": len(warm), "warm_ok": len(ok_w),
        "excludes": "VM boot, image pull, container start (local backend, process driver; the agent start "
                    "of every fresh instance is included)",
        "errors": errors[:5], "fresh": fresh, "warm": warm,
    }


def _d(t: dict, k: str, base: float):
    return round(t[k] - base, 4) if k in t else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=5, help="fresh-instance runs (the cold-start p50)")
    ap.add_argument("--warm-runs", type=int, default=4, help="runs reusing the idle instance")
    ap.add_argument("--timeout", type=float, default=120)
    ap.add_argument("--gpu", choices=("auto", "yes", "no"), default="auto")
    a = ap.parse_args()
    r = measure_cold_start(a.runs, a.warm_runs, a.timeout, gpu=a.gpu)
    print(json.dumps(r))
    return 0 if r["fresh_ok"] == r["fresh_runs"] and r["warm_ok"] == r["warm_runs"] else 1


if __name__ == "__main__":
    sys.exit(main())
