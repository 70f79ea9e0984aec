"""Background reconcilers driven directly against the DB with mocked backends/agents (reference:
``src/tests/_internal/server/background/tasks/test_process_{instances,submitted_jobs,runs,
running_jobs,terminating_jobs}.py``): unreachable hosts, idle timeout, termination retries,
no-capacity failures and the retry policy, runner unreachability."""

from datetime import timedelta
from unittest import mock

import pytest

from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.instances import (
    Disk,
    Gpu,
    InstanceAvailability,
    InstanceOfferWithAvailability,
    InstanceStatus,
    InstanceType,
    Resources,
)
from dstack_amd.core.models.runs import (
    JobProvisioningData,
    JobStatus,
    JobTerminationReason,
    RunSpec,
    RunStatus,
)
from dstack_amd.server.db import session_scope
from dstack_amd.server.models import InstanceModel, JobModel, ProjectModel, RunModel, UserModel
from dstack_amd.server.services import pools as pools_services
from dstack_amd.utils.common import get_current_datetime


def _itype(gpus=8):
    return InstanceType(name="8xMI355X", resources=Resources(cpus=128, memory_mib=2048 * 1024,
                                                             gpus=[Gpu(name="MI355X", memory_mib=288 * 1024)] * gpus,
                                                             disk=Disk(size_mib=1024 * 1024)))


def _jpd(backend=BackendType.AWS):
    return JobProvisioningData(backend=backend, instance_type=_itype(), instance_id="i-1", hostname="1.2.3.4",
                               internal_ip="10.0.0.1", region="us-east-1", price=10.0, username="ubuntu",
                               ssh_port=22, dockerized=True)


def _instance(s, status=InstanceStatus.IDLE, backend=BackendType.AWS, **kw):
    project = s.query(ProjectModel).filter_by(name="main").one()
    pool = pools_services.get_or_create_default_pool(s, project)
    offer = InstanceOfferWithAvailability(backend=backend, instance=_itype(), region="us-east-1", price=10.0,
                                          availability=InstanceAvailability.AVAILABLE)
    inst = pools_services.create_instance_model(
        s, project, pool, name=f"inst-{status.value}", status=status, backend=backend.value, region="us-east-1",
        price=10.0, job_provisioning_data=_jpd(backend).model_dump_json(), offer=offer.model_dump_json(),
        total_blocks=1, busy_blocks=0, started_at=get_current_datetime(), **kw)
    return inst.id


def _at(delta: timedelta):
    """Patch the reconcilers' clock forward by ``delta``."""
    now = get_current_datetime() + delta
    return mock.patch("dstack_amd.server.background.tasks.process_instances.get_current_datetime", return_value=now)


# ---- instances --------------------------------------------------------------------------------
def test_unreachable_instance_terminated_after_deadline(db):
    from dstack_amd.server.background.tasks import process_instances as pi

    with session_scope() as s:
        iid = _instance(s)
    with mock.patch.object(pi, "get_shim_client", side_effect=ConnectionError("down")):
        with session_scope() as s:
            pi._process_instance(s, iid)
        with session_scope() as s:
            inst = s.get(InstanceModel, iid)
            assert inst.unreachable and inst.status == "idle" and inst.termination_deadline is not None
        with _at(timedelta(minutes=21)), session_scope() as s:
            pi._process_instance(s, iid)
    with session_scope() as s:
        inst = s.get(InstanceModel, iid)
        assert inst.status == "terminating" and inst.termination_reason == "unreachable"


def test_reachable_again_clears_deadline(db):
    from dstack_amd.server.background.tasks import process_instances as pi

    with session_scope() as s:
        iid = _instance(s)
    with mock.patch.object(pi, "get_shim_client", side_effect=ConnectionError("down")), session_scope() as s:
        pi._process_instance(s, iid)
    ok = mock.Mock()
    ok.healthcheck.return_value = {"service": "dstack-shim"}
    with mock.patch.object(pi, "get_shim_client", return_value=ok), session_scope() as s:
        pi._process_instance(s, iid)
    with session_scope() as s:
        inst = s.get(InstanceModel, iid)
        assert not inst.unreachable and inst.termination_deadline is None


def test_idle_instance_terminated_after_idle_duration(db):
    from dstack_amd.server.background.tasks import process_instances as pi

    ok = mock.Mock()
    ok.healthcheck.return_value = {"service": "dstack-shim"}
    with session_scope() as s:
        iid = _instance(s, termination_idle_time=300)
    with mock.patch.object(pi, "get_shim_client", return_value=ok):
        with _at(timedelta(seconds=60)), session_scope() as s:
            pi._process_instance(s, iid)
        with session_scope() as s:
            assert s.get(InstanceModel, iid).status == "idle"
        with _at(timedelta(seconds=400)), session_scope() as s:
            pi._process_instance(s, iid)
    with session_scope() as s:
        inst = s.get(InstanceModel, iid)
        assert inst.status == "terminating" and inst.termination_reason == "idle timeout"


def test_termination_retried_then_given_up(db):
    from dstack_amd.server.background.tasks import process_instances as pi

    with session_scope() as s:
        iid = _instance(s, status=InstanceStatus.TERMINATING)
    compute = mock.Mock()
    compute.terminate_instance.side_effect = RuntimeError("cloud API 500")
    with mock.patch.object(pi.backends_services, "get_project_backend", return_value=compute):
        with session_scope() as s:
            pi._process_instance(s, iid)
        with session_scope() as s:
            assert s.get(InstanceModel, iid).status == "terminating"  # will retry
        with _at(timedelta(minutes=16)), session_scope() as s:
            pi._process_instance(s, iid)
    with session_scope() as s:
        inst = s.get(InstanceModel, iid)
        assert inst.status == "terminated" and inst.deleted
    assert compute.terminate_instance.call_count == 2


def test_provisioning_instance_becomes_idle_when_shim_answers(db):
    from dstack_amd.server.background.tasks import process_instances as pi

    with session_scope() as s:
        iid = _instance(s, status=InstanceStatus.PROVISIONING)
    ok = mock.Mock()
    ok.healthcheck.return_value = {"service": "dstack-shim"}
    with mock.patch.object(pi, "get_shim_client", return_value=ok), session_scope() as s:
        pi._process_instance(s, iid)
    with session_scope() as s:
        assert s.get(InstanceModel, iid).status == "idle"


@pytest.mark.parametrize("busy_blocks,want", [(0, "idle"), (1, "busy")])
def test_provisioning_ready_clears_health_and_deadline(db, busy_blocks, want):
    """(reference: ``test_check_shim_transitions_provisioning_on_ready`` / ``_on_busy``) a host that
    had health problems while provisioning comes up clean; a job already assigned makes it BUSY."""
    from datetime import timedelta

    from dstack_amd.server.background.tasks import process_instances as pi

    with session_scope() as s:
        iid = _instance(s, status=InstanceStatus.PROVISIONING)
        inst = s.get(InstanceModel, iid)
        inst.health_status = "ssh connect problem"
        inst.termination_deadline = get_current_datetime() + timedelta(days=1)
        inst.busy_blocks = busy_blocks
    ok = mock.Mock()
    ok.healthcheck.return_value = {"service": "dstack-shim"}
    with mock.patch.object(pi, "get_shim_client", return_value=ok), session_scope() as s:
        pi._process_instance(s, iid)
    with session_scope() as s:
        inst = s.get(InstanceModel, iid)
        assert (inst.status, inst.health_status, inst.termination_deadline) == (want, None, None)


def test_provisioning_unreachable_times_out(db):
    """(reference: ``test_check_shim_transitions_provisioning_on_terminating``) the shim never
    answers: the health status says so, and past the provisioning deadline the host terminates."""
    from dstack_amd.server.background.tasks import process_instances as pi

    with session_scope() as s:
        iid = _instance(s, status=InstanceStatus.PROVISIONING)
        s.get(InstanceModel, iid).started_at = get_current_datetime() - pi.PROVISIONING_DEADLINE / 2
    down = mock.Mock()
    down.healthcheck.side_effect = ConnectionError("ssh: connect to host: timed out")
    with mock.patch.object(pi, "get_shim_client", return_value=down), session_scope() as s:
        pi._process_instance(s, iid)
    with session_scope() as s:
        inst = s.get(InstanceModel, iid)
        assert inst.status == "provisioning" and inst.health_status
        inst.started_at = get_current_datetime() - pi.PROVISIONING_DEADLINE * 2
    with mock.patch.object(pi, "get_shim_client", return_value=down), session_scope() as s:
        pi._process_instance(s, iid)
    with session_scope() as s:
        inst = s.get(InstanceModel, iid)
        assert inst.status == "terminating" and inst.termination_reason == "provisioning timeout"
        assert inst.termination_deadline is not None


# ---- submitted jobs / runs --------------------------------------------------------------------
def _submit(s, conf: dict, name="r1"):
    from dstack_amd.server.services import runs as runs_services

    project = s.query(ProjectModel).filter_by(name="main").one()
    user = s.query(UserModel).filter_by(name="admin").one()
    spec = RunSpec.model_validate({"run_name": name, "repo_id": "virt", "repo_data": {"repo_type": "virtual"},
                                   "configuration": conf, "ssh_key_pub": ""})
    return runs_services.submit_run(s, project, user, spec).id


def _job(s, run_id):
    return s.query(JobModel).filter_by(run_id=run_id).order_by(JobModel.submission_num.desc()).first()


def test_no_offers_fails_job_with_no_capacity(db):
    from dstack_amd.server.background.tasks import process_submitted_jobs as psj

    with session_scope() as s:
        rid = _submit(s, {"type": "task", "commands": ["x"], "resources": {"gpu": "MI355X:8"}})
    with mock.patch.object(psj.offers_services, "get_offers_by_requirements", return_value=[]), session_scope() as s:
        psj._process_job(s, _job(s, rid).id)
    with session_scope() as s:
        j = _job(s, rid)
        assert j.status in ("terminating", "failed")
        assert j.termination_reason == JobTerminationReason.FAILED_TO_START_DUE_TO_NO_CAPACITY.value


def test_idle_pool_instance_reused_with_xgmi_gpus(db):
    from dstack_amd.server.background.tasks import process_submitted_jobs as psj

    with session_scope() as s:
        iid = _instance(s, backend=BackendType.REMOTE)
        inst = s.get(InstanceModel, iid)
        from dstack_amd.core.models.instances import GpuDevice, HostTopology

        x = [[0 if a == b else 1 for b in range(8)] for a in range(8)]
        inst.host_topology = HostTopology(gpus=[GpuDevice(index=i, name="MI355X") for i in range(8)], xgmi=x,
                                          numa={i: i // 4 for i in range(8)}).model_dump_json()
        inst.total_blocks = 8
        rid = _submit(s, {"type": "task", "commands": ["x"], "resources": {"gpu": "MI355X:4"}})
    with session_scope() as s:
        psj._process_job(s, _job(s, rid).id)
    with session_scope() as s:
        j = _job(s, rid)
        inst = s.get(InstanceModel, iid)
        assert j.status == "provisioning" and j.instance_id == iid
        assert inst.status == "busy" and inst.busy_blocks == 4
        assert len(inst.busy_gpus.split(",")) == 4


def test_retry_policy_resubmits_after_no_capacity(db):
    from dstack_amd.server.background.tasks import process_runs as pr
    from dstack_amd.server.background.tasks import process_submitted_jobs as psj
    from dstack_amd.server.background.tasks import process_terminating_jobs as ptj

    with session_scope() as s:
        rid = _submit(s, {"type": "task", "commands": ["x"], "resources": {"gpu": "MI355X:8"},
                          "retry": {"on_events": ["no-capacity"], "duration": "1h"}})
    with mock.patch.object(psj.offers_services, "get_offers_by_requirements", return_value=[]), session_scope() as s:
        psj._process_job(s, _job(s, rid).id)
    with session_scope() as s:
        j = _job(s, rid)
        if j.status == "terminating":
            ptj._process_job(s, j.id)
    for _ in range(3):
        with session_scope() as s:
            pr._process_run(s, rid)
    with session_scope() as s:
        run = s.get(RunModel, rid)
        jobs = s.query(JobModel).filter_by(run_id=rid).all()
        # the run is not failed: it waits (pending) or already resubmitted a new job submission
        assert run.status in (RunStatus.PENDING.value, RunStatus.SUBMITTED.value), run.status
        assert not RunStatus(run.status).is_finished()
        assert len(jobs) >= 1


def test_runner_unreachable_interrupts_job(db):
    from dstack_amd.server.background.tasks import process_running_jobs as prj

    with session_scope() as s:
        iid = _instance(s)
        rid = _submit(s, {"type": "task", "commands": ["x"]})
        j = _job(s, rid)
        j.status = JobStatus.RUNNING.value
        j.instance_id = iid
        j.job_provisioning_data = _jpd().model_dump_json()
        jid = j.id
    with mock.patch.object(prj, "get_runner_client", side_effect=ConnectionError("runner gone")):
        with session_scope() as s:
            j = s.get(JobModel, jid)
            prj._process_running(s, j.run, j)
        later = get_current_datetime() + timedelta(minutes=15)
        with mock.patch.object(prj, "get_current_datetime", return_value=later), session_scope() as s:
            j = s.get(JobModel, jid)
            prj._process_running(s, j.run, j)
    with session_scope() as s:
        j = s.get(JobModel, jid)
        assert j.termination_reason == JobTerminationReason.INTERRUPTED_BY_NO_CAPACITY.value


@pytest.mark.parametrize("reason,retry_events,expect_retry", [
    (JobTerminationReason.INTERRUPTED_BY_NO_CAPACITY, ["interruption"], True),
    (JobTerminationReason.INTERRUPTED_BY_NO_CAPACITY, ["no-capacity"], False),
    (JobTerminationReason.FAILED_TO_START_DUE_TO_NO_CAPACITY, ["no-capacity"], True),
    (JobTerminationReason.CONTAINER_EXITED_WITH_ERROR, ["error"], True),
    (JobTerminationReason.CONTAINER_EXITED_WITH_ERROR, ["interruption"], False),
    (JobTerminationReason.TERMINATED_BY_USER, ["error", "interruption", "no-capacity"], False),
])
def test_retry_decision(db, reason, retry_events, expect_retry):
    """Which termination reasons count as which retry event (reference ``_should_retry_job``)."""
    from dstack_amd.server.background.tasks import process_runs as pr

    with session_scope() as s:
        rid = _submit(s, {"type": "task", "commands": ["x"], "retry": {"on_events": retry_events, "duration": "1h"}})
        j = _job(s, rid)
        j.status = JobStatus.FAILED.value
        j.termination_reason = reason.value
        j.finished_at = get_current_datetime()
        if reason != JobTerminationReason.FAILED_TO_START_DUE_TO_NO_CAPACITY:
            j.job_provisioning_data = _jpd().model_dump_json()  # it had been running
        s.flush()
        run = s.get(RunModel, rid)
        assert (pr._retry_duration(run, j) is not None) == expect_retry


def test_gpu_probe_result_recorded_as_instance_health(db):
    """The runner's dstack-probe document (pull response ``gpu_probe``) becomes the instance's
    health; a probe below thresholds marks the instance unhealthy."""
    from dstack_amd.server.background.tasks import process_running_jobs as prj

    with session_scope() as s:
        iid = _instance(s)
        rid = _submit(s, {"type": "task", "commands": ["x"]})
        j = _job(s, rid)
        j.status = JobStatus.RUNNING.value
        j.instance_id = iid
        j.job_provisioning_data = _jpd().model_dump_json()
        jid = j.id
    for doc, healthy in (({"hbm_tb_s": [6.05], "mfma_bf16_tflops": [2103.8], "healthy": True}, True),
                         ({"hbm_tb_s": [1.1], "mfma_bf16_tflops": [310.0], "healthy": False}, False)):
        runner = mock.Mock()
        runner.pull.return_value = {"job_states": [], "job_logs": [], "runner_logs": [], "last_updated": 1,
                                    "gpu_probe": doc}
        with mock.patch.object(prj, "get_runner_client", return_value=runner), session_scope() as s:
            j = s.get(JobModel, jid)
            prj._process_running(s, j.run, j)
        with session_scope() as s:
            inst = pools_services.instance_model_to_instance(s.get(InstanceModel, iid))
            assert inst.health is not None
            assert inst.health["healthy"] is healthy
            assert inst.health["hbm_tb_s"] == doc["hbm_tb_s"]
            assert (s.get(InstanceModel, iid).health_status is None) is healthy


def test_unhealthy_instance_not_reused(db):
    """An instance whose GPU probe failed is skipped when pool instances are matched to a job."""
    from dstack_amd.core.models.instances import InstanceHealth
    from dstack_amd.core.models.profiles import Profile
    from dstack_amd.core.models.resources import ResourcesSpec
    from dstack_amd.core.models.runs import Requirements

    with session_scope() as s:
        iid = _instance(s)
        inst = s.get(InstanceModel, iid)
        req = Requirements(resources=ResourcesSpec.model_validate({"gpu": "MI355X:8"}))
        assert [i.id for i, _ in pools_services.filter_pool_instances([inst], Profile(name="p"), req)] == [iid]
        inst.health_data = InstanceHealth(healthy=False, hbm_tb_s=[0.9]).model_dump_json()
        assert pools_services.filter_pool_instances([inst], Profile(name="p"), req) == []
