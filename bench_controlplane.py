#!/usr/bin/env python3
"""Control-plane capacity bench: the only numbers the reference publishes that compare like for like.

Reference (``src/dstack/_internal/server/background/__init__.py:39-46``): one server
replica handles **150 active jobs / runs / instances with up to 2 minutes of processing latency**,
and processes at most **75 submitted jobs / instances per minute**.

What this measures, on ONE server process (the real app: HTTP API, SQLite WAL, the event-driven
reconcilers on their worker threads):

* N idle SSH-fleet hosts (8x MI355X each) are registered; the shim and runner on every host are
  in-memory fakes that answer each call after ``--rpc-latency-ms`` (the SSH-tunnel + HTTP round
  trip a real agent costs) -- everything server-side is the production code path;
* N task runs are submitted over HTTP as fast as one client can;
* ``submit_to_running`` = per-job time from submission to RUNNING (runner accepted the job):
  p50/p99/max, and the throughput of submissions processed per minute;
* with all N running, ``processing latency`` = per-job interval between consecutive log/state pulls
  of the running-job reconciler (how stale a job's state can get): p50/p99/max over the hold;
* then every runner reports done: time until all jobs are finished and hosts idle again.

Prints one JSON line (``--out`` also writes it).  No GPU, no network: fakes stand in for the
agents, which is how the reference tests its reconcilers too.
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import tempfile
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def _pct(xs, p):
    if not xs:
        return None
    xs = sorted(xs)
    k = min(len(xs) - 1, max(0, int(round(p / 100.0 * (len(xs) - 1)))))
    return round(xs[k], 3)


class _Lat:
    def __init__(self, ms: float):
        self.s = ms / 1000.0

    def __call__(self):
        if self.s > 0:
            time.sleep(self.s)


class FakeShim:
    def __init__(self, lat):
        self.lat = lat
        self.tasks = {}
        self.lock = threading.Lock()

    def healthcheck(self):
        self.lat()
        return {"service": "dstack-shim"}

    def gpu_health(self):
        self.lat()
        return None

    def submit_task(self, body):
        self.lat()
        with self.lock:
            self.tasks[body["id"]] = {"id": body["id"], "status": "running", "runner_port": 10999,
                                      "ports": [{"container": 10999, "host": 10999}], "gpus": body.get("gpu_indices")}

    def get_task(self, task_id):
        self.lat()
        with self.lock:
            return dict(self.tasks[task_id]) if task_id in self.tasks else None

    def terminate_task(self, task_id, reason="", message="", timeout=10):
        self.lat()
        with self.lock:
            if task_id in self.tasks:
                self.tasks[task_id]["status"] = "terminated"

    def remove_task(self, task_id):
        self.lat()
        with self.lock:
            self.tasks.pop(task_id, None)


class FakeRunner:
    def __init__(self, lat, agents):
        self.lat = lat
        self.agents = agents
        self.pull_times = []
        self.started_at = None

    def healthcheck(self):
        self.lat()
        return {"service": "dstack-runner"}

    def submit_job(self, *a, **k):
        self.lat()

    def upload_code(self, code):
        self.lat()

    def run_job(self):
        self.lat()
        self.started_at = time.time()

    def stop(self):
        self.lat()

    def get_metrics(self):
        self.lat()
        return None

    def pull(self, timestamp, wait_ms=0):
        self.lat()
        self.pull_times.append(time.time())
        if self.agents.finish.is_set():
            return {"job_states": [{"state": "done", "exit_status": 0, "timestamp": 3}], "job_logs": [],
                    "runner_logs": [], "last_updated": 3000}
        if len(self.pull_times) == 1:
            return {"job_states": [{"state": "running", "timestamp": 1}],
                    "job_logs": [{"timestamp": int(time.time() * 1000), "message": "c3RhcnRlZAo="}],
                    "runner_logs": [], "last_updated": 1000}
        return {"job_states": [], "job_logs": [], "runner_logs": [], "last_updated": 1000 + len(self.pull_times)}


class Agents:
    def __init__(self, latency_ms):
        self.lat = _Lat(latency_ms)
        self.shims, self.runners = {}, {}
        self.lock = threading.Lock()
        self.finish = threading.Event()

    def shim(self, jpd, *a, **k):
        with self.lock:
            return self.shims.setdefault(jpd.hostname, FakeShim(self.lat))

    def runner(self, jpd, *a, **k):
        with self.lock:
            return self.runners.setdefault(jpd.hostname, FakeRunner(self.lat, self))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=150)
    ap.add_argument("--rpc-latency-ms", type=float, default=20.0,
                    help="per agent call (SSH tunnel + HTTP round trip of a real shim/runner)")
    ap.add_argument("--hold-s", type=float, default=30.0, help="how long all jobs stay running")
    ap.add_argument("--timeout-s", type=float, default=600.0)
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)

    tmp = tempfile.mkdtemp(prefix="dstack-cp-bench-")
    os.environ.update(DSTACK_DIR=os.path.join(tmp, "dstack"), DSTACK_SERVER_DIR=os.path.join(tmp, "server"),
                      DSTACK_SERVER_NO_CLIENT_CONFIG="1", DSTACK_SERVER_ADMIN_TOKEN="bench-token",
                      DSTACK_SERVER_LOG_LEVEL="WARNING")
    from unittest import mock

    from fastapi.testclient import TestClient

    from dstack_amd.core.models.backends import BackendType
    from dstack_amd.core.models.instances import (Disk, Gpu, InstanceAvailability, InstanceOfferWithAvailability,
                                                  InstanceStatus, InstanceType, Resources)
    from dstack_amd.core.models.runs import JobProvisioningData
    from dstack_amd.server.app import create_app
    from dstack_amd.server.background.tasks import process_instances as pi
    from dstack_amd.server.background.tasks import process_metrics as pm
    from dstack_amd.server.background.tasks import process_running_jobs as prj
    from dstack_amd.server.background.tasks import process_terminating_jobs as ptj
    from dstack_amd.server.db import session_scope
    from dstack_amd.server.models import InstanceModel, JobModel, ProjectModel
    from dstack_amd.server.services import pools as pools_services
    from dstack_amd.utils.common import get_current_datetime

    agents = Agents(args.rpc_latency_ms)
    patches = [mock.patch.object(prj, "get_shim_client", side_effect=agents.shim),
               mock.patch.object(prj, "get_runner_client", side_effect=agents.runner),
               mock.patch.object(ptj, "get_shim_client", side_effect=agents.shim),
               mock.patch.object(ptj, "get_runner_client", side_effect=agents.runner),
               mock.patch.object(pi, "get_shim_client", side_effect=agents.shim),
               mock.patch.object(pm, "get_runner_client", side_effect=agents.runner),
               mock.patch("dstack_amd.server.services.runner.client.get_runner_client", side_effect=agents.runner)]
    for p in patches:
        p.start()
    itype = InstanceType(name="8xMI355X", resources=Resources(
        cpus=128, memory_mib=2048 * 1024, gpus=[Gpu(name="MI355X", memory_mib=288 * 1024)] * 8,
        disk=Disk(size_mib=4 * 1024 * 1024)))
    result = {"metric": "control-plane capacity (submit->running, processing latency)", "jobs": args.jobs,
              "rpc_latency_ms": args.rpc_latency_ms,
              "reference": {"active_jobs": 150, "max_processing_latency_s": 120, "submissions_per_min": 75,
                            "source": "src/dstack/_internal/server/background/__init__.py:39-46"}}
    app = create_app(start_background=True)
    with TestClient(app) as c:
        c.headers.update({"Authorization": "Bearer bench-token"})
        with session_scope() as s:
            project = s.query(ProjectModel).filter_by(name="main").one()
            pool = pools_services.get_or_create_default_pool(s, project)
            for i in range(args.jobs):
                ip = f"10.{i // 65536}.{(i // 256) % 256}.{i % 256}"
                jpd = JobProvisioningData(backend=BackendType.REMOTE, instance_type=itype, instance_id=f"host-{i}",
                                          hostname=ip, internal_ip=ip, region="onprem", price=0.0, username="root",
                                          ssh_port=22, dockerized=True)
                offer = InstanceOfferWithAvailability(backend=BackendType.REMOTE, instance=itype, region="onprem",
                                                      price=0.0, availability=InstanceAvailability.AVAILABLE)
                pools_services.create_instance_model(
                    s, project, pool, name=f"host-{i}", status=InstanceStatus.IDLE, backend="remote", region="onprem",
                    price=0.0, job_provisioning_data=jpd.model_dump_json(), offer=offer.model_dump_json(),
                    total_blocks=1, busy_blocks=0, started_at=get_current_datetime(),
                    termination_policy="dont-destroy")
        # ---- submit N runs over HTTP ----
        conf = {"type": "task", "commands": ["python train.py"], "resources": {"gpu": "MI355X:8"}}
        t0 = time.time()
        submitted = {}
        for i in range(args.jobs):
            spec = {"run_name": f"bench-{i}", "repo_id": "bench", "repo_data": {"repo_type": "virtual"},
                    "configuration": conf, "ssh_key_pub": ""}
            r = c.post("/api/project/main/runs/submit", json={"run_spec": spec})
            if r.status_code != 200:
                raise SystemExit(f"submit failed: {r.status_code} {r.text[:300]}")
            submitted[f"bench-{i}"] = time.time()
        t_sub = time.time() - t0
        result["submit_api_s"] = round(t_sub, 3)
        result["submit_api_per_min"] = round(args.jobs / t_sub * 60, 1)
        # ---- wait for every job to reach RUNNING ----
        deadline = time.time() + args.timeout_s
        running_at = {}
        while time.time() < deadline:
            with session_scope() as s:
                rows = s.query(JobModel.job_name, JobModel.status, JobModel.timings).all()
            for name, st, timings in rows:
                if name not in running_at and st == "running":
                    tm = json.loads(timings or "{}")
                    running_at[name] = tm.get("running") or time.time()
            if len(running_at) >= args.jobs:
                break
            time.sleep(0.2)
        lat = []
        for name, ts in running_at.items():
            sub = submitted.get(name.rsplit("-", 2)[0])  # job name = <run>-<job_num>-<replica_num>
            if sub is not None:
                lat.append(ts - sub)
        all_running = time.time() - t0
        result["running"] = len(running_at)
        result["submit_to_running_s"] = {"p50": _pct(lat, 50), "p99": _pct(lat, 99), "max": _pct(lat, 100)}
        result["all_running_after_s"] = round(all_running, 2)
        result["processed_per_min"] = round(len(running_at) / all_running * 60, 1) if all_running else None
        # ---- hold: processing latency of the running-job loop ----
        for r in agents.runners.values():
            r.pull_times.clear()
        time.sleep(args.hold_s)
        gaps, stale = [], []
        now = time.time()
        for r in agents.runners.values():
            pts = r.pull_times
            gaps += [b - a for a, b in zip(pts, pts[1:])]
            stale.append(now - pts[-1] if pts else args.hold_s)
        result["hold_s"] = args.hold_s
        result["pull_interval_s"] = {"p50": _pct(gaps, 50), "p99": _pct(gaps, 99), "max": _pct(gaps, 100)}
        result["max_staleness_s"] = round(max(stale), 2) if stale else None
        result["pulls_per_s"] = round(sum(len(r.pull_times) for r in agents.runners.values()) / args.hold_s, 1)
        # ---- every job finishes: drain ----
        agents.finish.set()
        t1 = time.time()
        while time.time() < deadline:
            with session_scope() as s:
                left = s.query(JobModel).filter(JobModel.status.notin_(["done", "failed", "terminated",
                                                                        "aborted"])).count()
                busy = s.query(InstanceModel).filter(InstanceModel.busy_blocks > 0).count()
            if left == 0 and busy == 0:
                break
            time.sleep(0.2)
        result["drain_s"] = round(time.time() - t1, 2)
        result["jobs_left"] = left
    for p in patches:
        p.stop()
    ok = (result["running"] == args.jobs and result["submit_to_running_s"]["max"] is not None
          and result["submit_to_running_s"]["max"] <= 120 and (result["max_staleness_s"] or 0) <= 120)
    result["within_reference_bounds"] = bool(ok)
    line = json.dumps(result)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
