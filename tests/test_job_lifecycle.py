"""Whole job lifecycle through the reconcilers with in-memory fake agents (reference test strategy:
``src/tests/_internal/server/background/tasks/test_process_{submitted,running,terminating}_jobs.py``
and ``test_process_runs.py`` — every background task called directly against the DB, the shim and
the runner replaced by objects that record what the server asked of them).

Covered: SUBMITTED -> PROVISIONING (pool instance, xGMI GPU pick) -> PULLING (shim task body:
GPUs, ports, keys) -> RUNNING (runner submit/upload/run, cluster info) -> logs pulled into storage
-> DONE/FAILED -> TERMINATING -> instance blocks and GPUs released -> run status; multinode
rendezvous (workers wait for the master, every rank gets the same ``ClusterInfo``); container
creation failure; non-zero exit; graceful stop; service replica registration."""

from __future__ import annotations

import itertools
import json
from typing import Dict, List, Optional
from unittest import mock

import pytest

from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.instances import (
    Disk,
    Gpu,
    GpuDevice,
    HostTopology,
    InstanceAvailability,
    InstanceOfferWithAvailability,
    InstanceStatus,
    InstanceType,
    Resources,
)
from dstack_amd.core.models.runs import JobProvisioningData, JobStatus, JobTerminationReason, RunSpec, RunStatus
from dstack_amd.server.background.tasks import process_running_jobs as prj
from dstack_amd.server.background.tasks import process_runs as pr
from dstack_amd.server.background.tasks import process_submitted_jobs as psj
from dstack_amd.server.background.tasks import process_terminating_jobs as ptj
from dstack_amd.server.db import session_scope
from dstack_amd.server.models import InstanceModel, JobModel, ProjectModel, RunModel, UserModel
from dstack_amd.server.services import pools as pools_services
from dstack_amd.server.services import runs as runs_services
from dstack_amd.utils.common import get_current_datetime

_ips = itertools.count(11)


# ---- fake agents ------------------------------------------------------------------------------
class FakeShim:
    """dstack-shim task API: submit_task / get_task / terminate_task / remove_task."""

    def __init__(self, host: str, fail_create: Optional[str] = None, ports_ready: bool = True):
        self.host = host
        self.tasks: Dict[str, dict] = {}
        self.submitted: List[dict] = []
        self.terminated: List[tuple] = []
        self.removed: List[str] = []
        self.fail_create = fail_create
        self.ports_ready = ports_ready  # bridge network: docker has published the container ports
        self.down = False  # the host stopped answering

    def healthcheck(self):
        return {"service": "dstack-shim"}

    def submit_task(self, body: dict):
        self.submitted.append(body)
        task = {"id": body["id"], "status": "running", "ports": [], "runner_port": None,
                "gpus": body.get("gpu_indices"), "network_mode": body.get("network_mode")}
        self._publish(task, body.get("ports") or [])
        if self.fail_create:
            task.update(status="terminated", termination_reason="creating_container_error",
                        termination_message=self.fail_create)
        self.tasks[body["id"]] = task

    def _publish(self, task: dict, ports: List[int]):
        """Like the real shim: host network -> the runner on its own port; bridge -> every
        container port (runner 10999, sshd 10022, the app's) published on a host port."""
        if task["network_mode"] != "bridge":
            task.update(runner_port=10999, ports=[{"container": 10999, "host": 10999}])
        elif self.ports_ready:
            cports = [10999, 10022] + list(ports)
            task["ports"] = [{"container": c, "host": 32000 + i} for i, c in enumerate(cports)]
            task["runner_port"] = 32000

    def get_task(self, task_id: str):
        if self.down:
            raise ConnectionError("ssh: connect to host: Connection timed out")
        task = self.tasks.get(task_id)
        if task is not None and not task["ports"] and task["status"] == "running":
            self._publish(task, [])
        return task

    def terminate_task(self, task_id, reason, message, timeout=10):
        self.terminated.append((task_id, reason))
        if task_id in self.tasks:
            self.tasks[task_id]["status"] = "terminated"

    def remove_task(self, task_id):
        self.removed.append(task_id)
        self.tasks.pop(task_id, None)


class FakeRunner:
    """dstack-runner API: the job ends with ``final_state`` after one pull that carries logs."""

    def __init__(self, final_state: str = "done", exit_status: int = 0):
        self.submitted = None
        self.code = None
        self.started = False
        self.stopped = False
        self.final_state = final_state
        self.exit_status = exit_status
        self.pulls = 0

    def healthcheck(self):
        return {"service": "dstack-runner"}

    def submit_job(self, run_spec, run_name, repo_data, job_spec, cluster, secrets, creds):
        self.submitted = {"run_name": run_name, "job_spec": job_spec, "cluster": cluster, "secrets": secrets}

    def upload_code(self, code):
        self.code = code

    def run_job(self):
        self.started = True

    def stop(self):
        self.stopped = True

    def pull(self, timestamp: int):
        self.pulls += 1
        if self.pulls == 1:
            return {"job_states": [{"state": "running", "timestamp": 1}],
                    "job_logs": [{"timestamp": 1000, "message": "aGVsbG8K"}],  # "hello\n"
                    "runner_logs": [], "last_updated": 1000}
        if self.final_state is None:
            return {"job_states": [], "job_logs": [], "runner_logs": [], "last_updated": 1000 + self.pulls}
        st = {"state": self.final_state, "timestamp": 2}
        if self.final_state == "failed":
            st.update(termination_reason="container_exited_with_error", exit_status=self.exit_status)
        elif self.final_state == "done":
            st.update(exit_status=0)
        return {"job_states": [st], "job_logs": [], "runner_logs": [], "last_updated": 2000}


class Agents:
    """Routes ``get_shim_client`` / ``get_runner_client`` to one fake per host."""

    def __init__(self, **runner_kw):
        self.shims: Dict[str, FakeShim] = {}
        self.runners: Dict[str, FakeRunner] = {}
        self.runner_kw = runner_kw
        self.fail_create: Optional[str] = None

    def shim(self, jpd, key=None, *a, **kw):
        if jpd.hostname not in self.shims:
            self.shims[jpd.hostname] = FakeShim(jpd.hostname, self.fail_create)
        return self.shims[jpd.hostname]

    def runner(self, jpd, jrd=None, key=None, *a, **kw):
        if jpd.hostname not in self.runners:
            self.runners[jpd.hostname] = FakeRunner(**self.runner_kw)
        return self.runners[jpd.hostname]

    def patch(self):
        return _Patches(self)


class _Patches:
    def __init__(self, agents: Agents):
        self.ps = [mock.patch.object(prj, "get_shim_client", side_effect=agents.shim),
                   mock.patch.object(prj, "get_runner_client", side_effect=agents.runner),
                   mock.patch.object(ptj, "get_shim_client", side_effect=agents.shim),
                   mock.patch.object(ptj, "get_runner_client", side_effect=agents.runner),
                   # stop_runner imports the client function at call time
                   mock.patch("dstack_amd.server.services.runner.client.get_runner_client",
                              side_effect=agents.runner)]

    def __enter__(self):
        for p in self.ps:
            p.start()
        return self

    def __exit__(self, *a):
        for p in reversed(self.ps):
            p.stop()


# ---- DB helpers -------------------------------------------------------------------------------
def _itype(n_gpus=8):
    return InstanceType(name="8xMI355X", resources=Resources(
        cpus=128, memory_mib=2048 * 1024, gpus=[Gpu(name="MI355X", memory_mib=288 * 1024)] * n_gpus,
        disk=Disk(size_mib=1024 * 1024)))


def _remote_instance(s, name: str, n_gpus: int = 8, blocks: int = 1) -> tuple:
    """An idle SSH-fleet host with 8 fully xGMI-connected MI355X (one block = whole host)."""
    ip = f"10.0.0.{next(_ips)}"
    project = s.query(ProjectModel).filter_by(name="main").one()
    pool = pools_services.get_or_create_default_pool(s, project)
    jpd = JobProvisioningData(backend=BackendType.REMOTE, instance_type=_itype(n_gpus), instance_id=name,
                              hostname=ip, internal_ip=ip, region="onprem", price=0.0, username="root",
                              ssh_port=22, dockerized=True)
    offer = InstanceOfferWithAvailability(backend=BackendType.REMOTE, instance=_itype(n_gpus), region="onprem",
                                          price=0.0, availability=InstanceAvailability.AVAILABLE)
    inst = pools_services.create_instance_model(
        s, project, pool, name=name, status=InstanceStatus.IDLE, backend="remote", region="onprem", price=0.0,
        job_provisioning_data=jpd.model_dump_json(), offer=offer.model_dump_json(), total_blocks=blocks,
        busy_blocks=0, started_at=get_current_datetime())
    x = [[0 if a == b else 1 for b in range(n_gpus)] for a in range(n_gpus)]
    inst.host_topology = HostTopology(gpus=[GpuDevice(index=i, name="MI355X") for i in range(n_gpus)], xgmi=x,
                                      numa={i: i // 4 for i in range(n_gpus)}).model_dump_json()
    s.flush()
    return inst.id, ip


def _submit(s, conf: dict, name: str = "run1") -> object:
    project = s.query(ProjectModel).filter_by(name="main").one()
    user = s.query(UserModel).filter_by(name="admin").one()
    spec = RunSpec.model_validate({"run_name": name, "repo_id": "virt", "repo_data": {"repo_type": "virtual"},
                                   "configuration": conf, "ssh_key_pub": "ssh-ed25519 AAAAuser"})
    return runs_services.submit_run(s, project, user, spec).id


def _jobs(s, run_id) -> List[JobModel]:
    return list(s.query(JobModel).filter_by(run_id=run_id).order_by(JobModel.replica_num, JobModel.job_num,
                                                                   JobModel.submission_num))


def _tick(run_id):
    """One pass of every job/run reconciler over this run, in the scheduler's order."""
    with session_scope() as s:
        ids = [(j.id, j.status) for j in _jobs(s, run_id)]
    for jid, st in ids:
        with session_scope() as s:
            if st == JobStatus.SUBMITTED.value:
                psj._process_job(s, jid)
    for jid, _ in ids:
        with session_scope() as s:
            prj._process_job(s, jid)
    for jid, _ in ids:
        with session_scope() as s:
            ptj._process_job(s, jid)
    with session_scope() as s:
        pr._process_run(s, run_id)


def _status(run_id):
    with session_scope() as s:
        run = s.get(RunModel, run_id)
        return run.status, [(j.status, j.termination_reason) for j in _jobs(s, run_id)]


def _run_to_end(run_id, max_ticks: int = 12):
    for _ in range(max_ticks):
        _tick(run_id)
        st, _ = _status(run_id)
        if RunStatus(st).is_finished():
            break
    return _status(run_id)


# ---- tests ------------------------------------------------------------------------------------
def test_single_node_task_runs_to_done_and_releases_gpus(db):
    agents = Agents()
    with session_scope() as s:
        iid, ip = _remote_instance(s, "node-a", blocks=8)  # 8 GPU blocks: a 4-GPU job takes half
        rid = _submit(s, {"type": "task", "commands": ["python train.py"], "image": "rocm/pytorch",
                          "resources": {"gpu": "MI355X:4"}, "ports": [6006]})
    with agents.patch():
        _tick(rid)  # SUBMITTED -> PROVISIONING (pool) -> PULLING -> RUNNING in one pass
        with session_scope() as s:
            (job,) = _jobs(s, rid)
            assert job.status == JobStatus.RUNNING.value, job.status
            inst = s.get(InstanceModel, iid)
            assert inst.status == InstanceStatus.BUSY.value and inst.busy_blocks == 4
            assert len(inst.busy_gpus.split(",")) == 4
            timings = job.timings
        shim = agents.shims[ip]
        body = shim.submitted[0]
        assert body["image_name"] == "rocm/pytorch" and body["gpu"] == 4
        assert len(body["gpu_indices"]) == 4 and 6006 in body["ports"]
        assert "ssh-ed25519 AAAAuser" in body["container_ssh_keys"]
        runner = agents.runners[ip]
        assert runner.started and runner.submitted["run_name"] == "run1"
        assert runner.submitted["cluster"].master_job_ip == ip and runner.submitted["cluster"].job_ips == [ip]
        assert timings  # cold-start stamps recorded
        status, jobs = _run_to_end(rid)
    assert status == RunStatus.DONE.value, (status, jobs)
    assert jobs == [(JobStatus.DONE.value, JobTerminationReason.DONE_BY_RUNNER.value)]
    assert shim.terminated and shim.removed  # container stopped and removed through the shim
    with session_scope() as s:
        inst = s.get(InstanceModel, iid)
        assert inst.status == InstanceStatus.IDLE.value and inst.busy_blocks == 0 and inst.busy_gpus == ""
        (job,) = _jobs(s, rid)
        assert job.exit_status == 0 and job.finished_at is not None


def test_job_logs_pulled_into_storage(db):
    from dstack_amd.server.services import logs as logs_services

    agents = Agents(final_state=None)  # keeps running
    with session_scope() as s:
        _remote_instance(s, "node-logs")
        rid = _submit(s, {"type": "task", "commands": ["echo hello"]})
    with agents.patch():
        _tick(rid)
        _tick(rid)
    with session_scope() as s:
        (job,) = _jobs(s, rid)
        job_id = str(job.id)
    got = logs_services.get_default_log_storage().poll_logs("main", "run1", job_id)
    assert [logs_services.decode_message(e) for e in got.logs] == ["hello\n"]


def test_nonzero_exit_fails_run_without_retry(db):
    agents = Agents(final_state="failed", exit_status=3)
    with session_scope() as s:
        _remote_instance(s, "node-b")
        rid = _submit(s, {"type": "task", "commands": ["exit 3"]})
    with agents.patch():
        status, jobs = _run_to_end(rid)
    assert status == RunStatus.FAILED.value
    assert jobs[-1] == (JobStatus.FAILED.value, JobTerminationReason.CONTAINER_EXITED_WITH_ERROR.value)
    with session_scope() as s:
        assert s.get(RunModel, rid).termination_reason == "job_failed"
        assert _jobs(s, rid)[-1].exit_status == 3


def test_nonzero_exit_retried_on_error_event(db):
    agents = Agents(final_state="failed", exit_status=1)
    with session_scope() as s:
        _remote_instance(s, "node-c")
        rid = _submit(s, {"type": "task", "commands": ["flaky"], "retry": {"on_events": ["error"], "duration": "1h"}})
    with agents.patch():
        for _ in range(4):
            _tick(rid)
        status, jobs = _status(rid)
        assert status == RunStatus.PENDING.value  # waits RETRY_DELAY before resubmitting
        assert jobs == [(JobStatus.FAILED.value, JobTerminationReason.CONTAINER_EXITED_WITH_ERROR.value)]
        later = get_current_datetime() + pr.RETRY_DELAY * 2
        with mock.patch.object(pr, "get_current_datetime", return_value=later):
            _tick(rid)
            assert _status(rid) == (RunStatus.SUBMITTED.value, [jobs[0], (JobStatus.SUBMITTED.value, None)])
            _tick(rid)  # the new submission lands on the (released) host again
    with session_scope() as s:
        run = s.get(RunModel, rid)
        subs = [(j.submission_num, j.status) for j in _jobs(s, rid)]
        assert run.status == RunStatus.RUNNING.value and run.resubmission_attempt == 1
        assert subs == [(0, JobStatus.FAILED.value), (1, JobStatus.RUNNING.value)], subs


def test_container_creation_failure_fails_job(db):
    agents = Agents()
    agents.fail_create = "image not found: rocm/nope"
    with session_scope() as s:
        iid, _ = _remote_instance(s, "node-d")
        rid = _submit(s, {"type": "task", "commands": ["x"], "image": "rocm/nope"})
    with agents.patch():
        status, jobs = _run_to_end(rid)
    assert status == RunStatus.FAILED.value
    assert jobs[-1] == (JobStatus.FAILED.value, JobTerminationReason.CREATING_CONTAINER_ERROR.value)
    with session_scope() as s:
        assert s.get(InstanceModel, iid).busy_blocks == 0


def test_multinode_rendezvous_cluster_info(db):
    """nodes: 2 — the worker waits for the master's host; both runners get the same ClusterInfo
    with the master first, and GPUs_per_job from the assigned GPUs."""
    agents = Agents(final_state=None)
    with session_scope() as s:
        _, ip_a = _remote_instance(s, "node-m0")
        _, ip_b = _remote_instance(s, "node-m1")
        rid = _submit(s, {"type": "task", "nodes": 2, "commands": ["torchrun train.py"],
                          "resources": {"gpu": "MI355X:8"}})
    with agents.patch():
        for _ in range(3):
            _tick(rid)
    with session_scope() as s:
        jobs = _jobs(s, rid)
        assert [j.status for j in jobs] == [JobStatus.RUNNING.value] * 2
        assert s.get(RunModel, rid).status == RunStatus.RUNNING.value
    clusters = [r.submitted["cluster"] for r in agents.runners.values()]
    assert len(clusters) == 2 and clusters[0] == clusters[1]
    c = clusters[0]
    assert len(c.job_ips) == 2 and set(c.job_ips) == {ip_a, ip_b} and c.gpus_per_job == 8
    master_runner = next(r for r in agents.runners.values() if r.submitted["job_spec"].job_num == 0)
    assert c.master_job_ip == c.job_ips[0]
    assert master_runner.submitted["job_spec"].jobs_per_replica == 2


def test_multinode_worker_waits_for_master(db):
    with session_scope() as s:
        rid = _submit(s, {"type": "task", "nodes": 2, "commands": ["x"]})
        jobs = _jobs(s, rid)
        worker = [j for j in jobs if j.job_num == 1][0].id
    with mock.patch.object(psj.offers_services, "get_offers_by_requirements", return_value=[]) as offers, \
            session_scope() as s:
        psj._process_job(s, worker)
        assert offers.call_count == 0  # no provisioning attempt before the master has a host
    with session_scope() as s:
        assert s.get(JobModel, worker).status == JobStatus.SUBMITTED.value


def test_graceful_stop_stops_runner_then_terminates(db):
    agents = Agents(final_state=None)
    with session_scope() as s:
        iid, ip = _remote_instance(s, "node-e")
        rid = _submit(s, {"type": "task", "commands": ["sleep infinity"]})
    with agents.patch():
        _tick(rid)
        with session_scope() as s:
            runs_services.stop_runs(s, s.get(RunModel, rid).project, ["run1"], abort=False)
        with session_scope() as s:
            pr._process_run(s, rid)  # TERMINATING run: stop the runner, delay removal
        assert agents.runners[ip].stopped
        with session_scope() as s:
            (job,) = _jobs(s, rid)
            assert job.status == JobStatus.TERMINATING.value and job.remove_at is not None
        later = get_current_datetime() + pr.RETRY_DELAY * 4
        with mock.patch.object(ptj, "get_current_datetime", return_value=later):
            with session_scope() as s:
                ptj._process_job(s, _jobs(s, rid)[0].id)
        with session_scope() as s:
            pr._process_run(s, rid)
    status, jobs = _status(rid)
    assert status == RunStatus.TERMINATED.value
    assert jobs[0] == (JobStatus.TERMINATED.value, JobTerminationReason.TERMINATED_BY_USER.value)
    with session_scope() as s:
        assert s.get(InstanceModel, iid).status == InstanceStatus.IDLE.value


def test_stop_is_not_overwritten_by_a_concurrent_run_pass(db):
    """A ``process_runs`` pass that loaded the run before the stop and commits a status transition
    after it must not write over TERMINATING: stop_runs waits for the pass to release the run."""
    import threading
    import time

    from dstack_amd.server.services.locking import lockset

    with session_scope() as s:
        rid = _submit(s, {"type": "task", "commands": ["sleep infinity"]})
        s.get(RunModel, rid).status = RunStatus.PROVISIONING.value
    loaded, done = threading.Event(), threading.Event()

    def background_pass():  # what claim_and_process + _process_active do, stretched out in time
        with lockset("runs").hold([rid]):
            with session_scope() as s:
                run = s.get(RunModel, rid)
                assert run.status == RunStatus.PROVISIONING.value
                loaded.set()
                time.sleep(0.3)  # the stop request arrives meanwhile
                run.status = RunStatus.RUNNING.value
        done.set()

    t = threading.Thread(target=background_pass)
    t.start()
    assert loaded.wait(5)
    with session_scope() as s:
        runs_services.stop_runs(s, s.get(RunModel, rid).project, ["run1"], abort=False)
    assert done.is_set()  # the stop waited for the pass instead of racing it
    t.join(5)
    with session_scope() as s:
        run = s.get(RunModel, rid)
        assert run.status == RunStatus.TERMINATING.value
        assert run.termination_reason == "stopped_by_user"


def test_fleet_delete_waits_for_a_concurrent_job_assignment(db):
    """An instance being assigned to a job (IDLE -> BUSY, committed after the assignment's flush)
    must not be terminated by a fleet delete that read it as IDLE: the delete waits and refuses."""
    import threading
    import time
    import uuid

    from dstack_amd.core.errors import ServerClientError
    from dstack_amd.server.models import FleetModel
    from dstack_amd.server.services import fleets as fleets_services
    from dstack_amd.server.services.locking import lockset, release_at_transaction_end

    with session_scope() as s:
        iid, _ = _remote_instance(s, "node-race")
        project = s.query(ProjectModel).filter_by(name="main").one()
        fleet = FleetModel(id=uuid.uuid4(), name="f-race", project_id=project.id, status="active", spec="{}")
        s.add(fleet)
        s.flush()
        s.get(InstanceModel, iid).fleet_id = fleet.id
    loaded = threading.Event()

    def assignment():  # _assign_pool_instance: lock, mark BUSY, flush; the job pass commits later
        ls = lockset("instances")
        assert ls.try_add_many([iid])
        with session_scope() as s:
            s.get(InstanceModel, iid).status = InstanceStatus.BUSY.value
            s.flush()
            release_at_transaction_end(s, ls, [iid])
            loaded.set()
            time.sleep(0.3)
            assert iid in ls  # still held between flush and commit
        assert iid not in ls  # released by the commit

    t = threading.Thread(target=assignment)
    t.start()
    assert loaded.wait(5)
    with pytest.raises(ServerClientError, match="busy"):
        with session_scope() as s:
            fleets_services.delete_fleets(s, s.query(ProjectModel).filter_by(name="main").one(), ["f-race"])
    t.join(5)
    with session_scope() as s:
        assert s.get(InstanceModel, iid).status == InstanceStatus.BUSY.value


def test_abort_skips_graceful_stop(db):
    agents = Agents(final_state=None)
    with session_scope() as s:
        _, ip = _remote_instance(s, "node-f")
        rid = _submit(s, {"type": "task", "commands": ["sleep infinity"]})
    with agents.patch():
        _tick(rid)
        with session_scope() as s:
            runs_services.stop_runs(s, s.get(RunModel, rid).project, ["run1"], abort=True)
        for _ in range(3):
            _tick(rid)
    assert not agents.runners[ip].stopped
    status, jobs = _status(rid)
    assert status == RunStatus.TERMINATED.value
    assert jobs[0] == (JobStatus.ABORTED.value, JobTerminationReason.ABORTED_BY_USER.value)


def test_service_replica_registered_when_running(db):
    agents = Agents(final_state=None)
    with session_scope() as s:
        _remote_instance(s, "node-g")
        rid = _submit(s, {"type": "service", "commands": ["python -m http.server 8000"], "port": 8000,
                          "gateway": False}, name="svc1")
    with agents.patch(), mock.patch("dstack_amd.server.services.services.register_replica") as reg:
        _tick(rid)
    assert reg.call_count == 1
    body = next(iter(agents.shims.values())).submitted[0]
    assert 8000 in body["ports"]


@pytest.mark.parametrize("blocks,gpus_per_job,jobs", [(8, 1, 8), (4, 2, 4), (2, 4, 2)])
def test_blocks_share_one_host_disjoint_gpus(db, blocks, gpus_per_job, jobs):
    """A host split into GPU blocks runs several jobs at once, each on its own xGMI-picked GPUs."""
    agents = Agents(final_state=None)
    with session_scope() as s:
        iid, _ = _remote_instance(s, "node-blocks", blocks=blocks)
        rids = [_submit(s, {"type": "task", "commands": ["x"], "resources": {"gpu": f"MI355X:{gpus_per_job}"}},
                        name=f"b{i}") for i in range(jobs)]
    with agents.patch():
        for rid in rids:
            _tick(rid)
    with session_scope() as s:
        inst = s.get(InstanceModel, iid)
        assert inst.busy_blocks == jobs and inst.status == InstanceStatus.BUSY.value
        picked = []
        for rid in rids:
            (job,) = _jobs(s, rid)
            assert job.status == JobStatus.RUNNING.value
            from dstack_amd.server.services import jobs as jobs_services

            picked.append(tuple(jobs_services.job_jrd(job).gpu_indices))
    flat = [g for p in picked for g in p]
    assert len(flat) == len(set(flat)) == jobs * gpus_per_job


def test_bridge_job_waits_for_published_runner_port(db):
    """Blocks put a job on a bridge network: the runner is reachable only through the host port
    docker publishes for it, so the job stays PULLING (runner not contacted) until the shim
    reports that mapping (reference: ``test_pulling_shim_port_mapping_not_ready``)."""
    agents = Agents()
    with session_scope() as s:
        iid, ip = _remote_instance(s, "node-b", blocks=2)
        rid = _submit(s, {"type": "task", "commands": ["true"], "resources": {"gpu": "MI355X:4"}})
    agents.shims[ip] = FakeShim(ip, ports_ready=False)
    with agents.patch():
        _tick(rid)
        with session_scope() as s:
            (job,) = _jobs(s, rid)
            assert job.status == JobStatus.PULLING.value
        assert ip not in agents.runners  # runner never contacted without its port
        agents.shims[ip].ports_ready = True
        _tick(rid)
        with session_scope() as s:
            (job,) = _jobs(s, rid)
            assert job.status == JobStatus.RUNNING.value
            from dstack_amd.server.services import jobs as jobs_services

            assert jobs_services.job_jrd(job).ports[10999] == 32000


def test_host_lost_while_pulling_interrupts_job(db):
    """The shim stops answering while the job is PULLING: after the unreachable grace the job is
    interrupted with no capacity (reference: ``test_pulling_shim_failed``), so retry can resubmit."""
    from datetime import timedelta

    from dstack_amd.server import settings

    agents = Agents()
    with session_scope() as s:
        iid, ip = _remote_instance(s, "node-c", blocks=2)
        rid = _submit(s, {"type": "task", "commands": ["true"], "resources": {"gpu": "MI355X:4"}})
    agents.shims[ip] = FakeShim(ip, ports_ready=False)
    with agents.patch():
        _tick(rid)
        agents.shims[ip].down = True
        _tick(rid)
        with session_scope() as s:
            (job,) = _jobs(s, rid)
            assert job.status == JobStatus.PULLING.value  # inside the grace period
        later = get_current_datetime() + timedelta(seconds=settings.DEFAULT_RUNNER_TIMEOUT)
        with mock.patch.object(prj, "get_current_datetime", return_value=later):
            _tick(rid)
        with session_scope() as s:
            (job,) = _jobs(s, rid)
            assert job.status in (JobStatus.TERMINATING.value, JobStatus.FAILED.value)
            assert job.termination_reason == JobTerminationReason.INTERRUPTED_BY_NO_CAPACITY.value


class _PreflightRunner(FakeRunner):
    """Runner of a 2-node job with DSTACK_RCCL_PREFLIGHT: the worker's pre-flight fails (a rank of the
    all-reduce timed out) before the job starts, the master's passes and keeps the job running."""

    def pull(self, timestamp: int):
        node = self.submitted["job_spec"].job_num
        if node == 1:
            doc = {"rccl_world": 16, "rccl_busbw_gb_s": None, "healthy": False, "message": "RCCL: rank 9 timed out"}
            st = {"state": "failed", "timestamp": 2, "termination_reason": "executor_error",
                  "termination_message": "RCCL pre-flight failed (exit 1): RCCL: rank 9 timed out"}
            return {"job_states": [st], "job_logs": [], "runner_logs": [], "last_updated": 2000,
                    "rccl_preflight": doc}
        doc = {"rccl_world": 16, "rccl_busbw_gb_s": 311.5, "healthy": True, "message": ""}
        st = {"state": "terminated", "timestamp": 3, "termination_reason": "terminated_by_user"} if self.stopped \
            else {"state": "running", "timestamp": 1}
        return {"job_states": [st], "job_logs": [], "runner_logs": [], "last_updated": 1000, "rccl_preflight": doc}


class _PreflightAgents(Agents):
    def runner(self, jpd, jrd=None, key=None, *a, **kw):
        if jpd.hostname not in self.runners:
            self.runners[jpd.hostname] = _PreflightRunner()
        return self.runners[jpd.hostname]


def test_rccl_preflight_failure_on_one_node_fails_the_replica(db):
    """A failed RCCL pre-flight on node 1 of a 2-node task fails that job with the probe's message,
    the run fails (job_failed) and terminates the master's job too; the failing host is marked
    unhealthy (no new jobs land on it) and the passing host records its bus bandwidth."""
    agents = _PreflightAgents()
    with session_scope() as s:
        ids = [_remote_instance(s, "node-p0")[0], _remote_instance(s, "node-p1")[0]]
        rid = _submit(s, {"type": "task", "nodes": 2, "commands": ["torchrun train.py"],
                          "resources": {"gpu": "MI355X:8"}, "env": {"DSTACK_RCCL_PREFLIGHT": "1"}})
    with agents.patch():
        status, jobs = _run_to_end(rid, max_ticks=6)
        # the master's job is stopped through its runner, then removed after the grace delay
        later = get_current_datetime() + pr.RETRY_DELAY * 4
        with mock.patch.object(ptj, "get_current_datetime", return_value=later):
            status, jobs = _run_to_end(rid, max_ticks=3)
    assert status == RunStatus.FAILED.value, (status, jobs)
    with session_scope() as s:
        run = s.get(RunModel, rid)
        assert run.termination_reason == "job_failed"
        assert all(r.stopped for r in agents.runners.values() if r.submitted["job_spec"].job_num == 0)
        by_num = {j.job_num: j for j in _jobs(s, rid)}
        worker, master = by_num[1], by_num[0]
        assert worker.status == JobStatus.FAILED.value
        assert worker.termination_reason == JobTerminationReason.EXECUTOR_ERROR.value
        assert "rank 9 timed out" in (worker.termination_reason_message or "")
        assert JobStatus(master.status).is_finished() and master.status != JobStatus.DONE.value
        insts = [s.get(InstanceModel, i) for i in ids]
        health = {i.name: json.loads(i.health_data) for i in insts}
        bad = [i for i in insts if not health[i.name]["healthy"]]
        good = [i for i in insts if health[i.name]["healthy"]]
        assert len(bad) == 1 and len(good) == 1
        assert "rank 9 timed out" in health[bad[0].name]["message"] and "RCCL pre-flight" in bad[0].health_status
        assert health[good[0].name]["rccl_busbw_gb_s"] == 311.5 and good[0].health_status is None
        # the scheduler no longer offers the failed host
        from dstack_amd.core.models.profiles import Profile
        from dstack_amd.core.models.resources import ResourcesSpec
        from dstack_amd.core.models.runs import Requirements

        picked = pools_services.filter_pool_instances(insts, Profile(name="p"), Requirements(resources=ResourcesSpec()))
        assert [i.name for i, _ in picked] == [good[0].name]
    # the job spec carried the opt-in to the runners
    assert all(r.submitted["job_spec"].env.get("DSTACK_RCCL_PREFLIGHT") == "1" for r in agents.runners.values())


def test_rccl_preflight_bandwidth_floor_ignores_concurrent_measurements(monkeypatch):
    """The DSTACK_RCCL_MIN_BUSBW_GB_S floor marks a host unhealthy only for a blocking
    (uncontended) pre-flight; a concurrent probe shared the GPUs with the job's start-up, so its
    low number is recorded but the host stays healthy.  A failed probe is unhealthy either way."""
    from types import SimpleNamespace

    monkeypatch.setenv("DSTACK_RCCL_MIN_BUSBW_GB_S", "200")

    def rec(doc):
        job = SimpleNamespace(instance=SimpleNamespace(health_data=None, health_status=None, name="h"))
        prj._record_rccl_preflight(job, doc)
        return json.loads(job.instance.health_data), job.instance.health_status

    h, st = rec({"rccl_busbw_gb_s": 90.0, "healthy": True, "mode": "concurrent"})
    assert h["healthy"] and h["rccl_busbw_gb_s"] == 90.0 and st is None
    h, st = rec({"rccl_busbw_gb_s": 90.0, "healthy": True, "mode": "blocking"})
    assert not h["healthy"] and "below 200.0" in st
    h, st = rec({"rccl_busbw_gb_s": 90.0, "healthy": True})  # older runners: treated as blocking
    assert not h["healthy"]
    h, st = rec({"rccl_busbw_gb_s": None, "healthy": False, "message": "rank 3 timed out", "mode": "concurrent"})
    assert not h["healthy"] and "rank 3 timed out" in st
