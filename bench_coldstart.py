"""Job cold-start benchmark: the first half of BASELINE's headline metric ("p50 job cold-start (s)").

Starts a real dstack-amd server (local backend: native ``dstack-shim`` process driver +
``dstack-runner``), then ``apply``s ``--runs`` tasks one after another through the public API and
reads each job's stage timestamps:

* ``submit_to_running``   : API submit  -> runner started the user command
* ``submit_to_first_log`` : API submit  -> first byte of job output (runner clock)

The first run includes instance creation (a cold host); the others reuse the idle instance as in
the reference's pool semantics.  p50 is over all runs.  The task itself is a trivial command so the
number measures the control plane, not the workload.
"""

from __future__ import annotations

import argparse
import json
import statistics
import sys
import time


def measure_cold_start(runs: int = 5, timeout: float = 120.0, command: str = "echo ready") -> dict:
    from dstack_amd.api import Task
    from dstack_amd.server.testing import ServerProcess

    samples = []
    with ServerProcess() as srv:
        client = srv.client()
        for i in range(runs):
            conf = Task(commands=[command], name=f"coldstart-{i}")
            t0 = time.time()
            run = client.runs.submit(conf)
            run.wait(timeout=timeout, poll=0.05)
            sub = run.model.jobs[0].job_submissions[-1]
            t = sub.timings or {}
            sub_ts = t.get("submitted", t0)
            sample = {
                "status": sub.status.value,
                "termination_reason": sub.termination_reason.value if sub.termination_reason else None,
                "message": sub.termination_reason_message,
                "submit_to_provisioned": _d(t, "provisioned", sub_ts) or _d(t, "assigned", sub_ts),
                "submit_to_running": _d(t, "running", sub_ts),
                "submit_to_first_log": _d(t, "first_log", sub_ts),
                "client_wall_to_done": time.time() - t0,
            }
            samples.append(sample)
            if sample["submit_to_first_log"] is None:
                print(f"coldstart run {i} failed: {sample}", file=sys.stderr)
                print(srv.log()[-4000:], file=sys.stderr)
                for chunk in run.logs(diagnose=True):
                    sys.stderr.write(chunk.decode(errors="replace"))
    ok = [s for s in samples if s["submit_to_first_log"] is not None]
    p50 = statistics.median([s["submit_to_first_log"] for s in ok]) if ok else None
    return {
        "cold_start_p50_s": p50,
        "running_p50_s": statistics.median([s["submit_to_running"] for s in ok]) if ok else None,
        "first_run_s": samples[0]["submit_to_first_log"] if samples else None,
        "runs": len(samples), "ok": len(ok), "samples": samples,
    }


def _d(t: dict, k: str, base: float):
    return round(t[k] - base, 4) if k in t else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--timeout", type=float, default=120)
    a = ap.parse_args()
    r = measure_cold_start(a.runs, a.timeout)
    print(json.dumps(r))
    return 0 if r["ok"] == r["runs"] else 1


if __name__ == "__main__":
    sys.exit(main())
