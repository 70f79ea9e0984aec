"""Background reconcilers, case by case against the reference's ``background/tasks/test_process_*.py``
where the other test files here do not already cover the case (mapping: ``docs/reference/
test-parity.md``): fleet garbage collection, gateway provisioning / connection, instance termination
retries, placement-group cleanup, runner liveness while provisioning, jobs with no backends, volume
provisioning, and termination of jobs on shared (blocks) instances."""

from __future__ import annotations

import json
import uuid
from datetime import timedelta
from unittest import mock

from sqlalchemy import select

from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.instances import InstanceStatus
from dstack_amd.core.models.runs import JobStatus, JobTerminationReason
from dstack_amd.server.db import session_scope
from dstack_amd.server.models import (
    FleetModel,
    GatewayModel,
    InstanceModel,
    JobModel,
    PlacementGroupModel,
    ProjectModel,
    RunModel,
    VolumeModel,
    volumes_attachments,
)
from dstack_amd.utils.common import get_current_datetime
from tests.test_reconcilers import _at, _instance, _job, _jpd, _submit


# ---- process_fleets -----------------------------------------------------------------------------
def _fleet(s, name, autocreated=False, status="active", nodes=None):
    project = s.query(ProjectModel).filter_by(name="main").one()
    conf = {"type": "fleet", "name": name}
    if nodes is not None:
        conf["nodes"] = nodes
    f = FleetModel(id=uuid.uuid4(), name=name, project_id=project.id, status=status,
                   spec=json.dumps({"configuration": conf, "profile": {"name": "default"},
                                    "autocreated": autocreated}),
                   created_at=get_current_datetime(), last_processed_at=get_current_datetime())
    s.add(f)
    s.flush()
    return f.id


def _process_fleet(fid):
    from dstack_amd.server.background.tasks import process_fleets as pf

    with session_scope() as s:
        pf._process_fleet(s, fid)
    with session_scope() as s:
        return s.get(FleetModel, fid)


def test_fleets_deletes_empty_autocreated_fleet(db):
    with session_scope() as s:
        fid = _fleet(s, "auto", autocreated=True)
    f = _process_fleet(fid)
    assert f.deleted and f.status == "terminated"


def test_fleets_deletes_terminating_user_fleet_once_empty(db):
    with session_scope() as s:
        fid = _fleet(s, "mine", status="terminating")
        iid = _instance(s, status=InstanceStatus.TERMINATING)
        s.get(InstanceModel, iid).fleet_id = fid
    assert not _process_fleet(fid).deleted  # its instance is still terminating
    with session_scope() as s:
        s.get(InstanceModel, iid).status = InstanceStatus.TERMINATED.value
    f = _process_fleet(fid)
    assert f.deleted and f.status == "terminated"


def test_fleets_keeps_fleet_with_active_run(db):
    with session_scope() as s:
        fid = _fleet(s, "used", autocreated=True)
        rid = _submit(s, {"type": "task", "commands": ["x"]}, name="user-of-fleet")
        s.get(RunModel, rid).fleet_id = fid
    assert not _process_fleet(fid).deleted
    with session_scope() as s:
        s.get(RunModel, rid).status = "done"
    assert _process_fleet(fid).deleted


def test_fleets_keeps_empty_user_fleet_with_zero_min_nodes(db):
    with session_scope() as s:
        fid = _fleet(s, "elastic", nodes={"min": 0, "max": 4})
    assert not _process_fleet(fid).deleted


# ---- gateways -----------------------------------------------------------------------------------
def _gateway(s, status="submitted", backend="aws"):
    from dstack_amd.server.models import BackendModel

    project = s.query(ProjectModel).filter_by(name="main").one()
    b = BackendModel(id=uuid.uuid4(), project_id=project.id, type=backend, config="{}", auth="{}")
    s.add(b)
    s.flush()
    conf = {"type": "gateway", "name": "gw", "backend": backend, "region": "us-east-1", "domain": "gw.example.com"}
    g = GatewayModel(id=uuid.uuid4(), name="gw", region="us-east-1", wildcard_domain="gw.example.com",
                     configuration=json.dumps(conf), status=status, project_id=project.id, backend_id=b.id,
                     created_at=get_current_datetime(), last_processed_at=get_current_datetime())
    s.add(g)
    s.flush()
    return g.id


def _gpd():
    from dstack_amd.core.models.gateways import GatewayProvisioningData

    return GatewayProvisioningData(instance_id="i-gw", ip_address="203.0.113.7", region="us-east-1",
                                   hostname="203.0.113.7", backend_data=json.dumps({"ssh_user": "ubuntu"}))


def test_gateways_provisions_and_connects(db):
    from dstack_amd.server import background
    from dstack_amd.server.services import backends as backends_services
    from dstack_amd.server.services import gateways as gateways_services

    with session_scope() as s:
        gid = _gateway(s)
    compute = mock.Mock()
    compute.create_gateway.return_value = _gpd()
    calls = []
    with mock.patch.object(backends_services, "get_project_backend", return_value=compute), \
            mock.patch.object(gateways_services, "_call", side_effect=lambda g, m, p, b=None: calls.append(p) or {}):
        background.process_submitted_gateways()
    with session_scope() as s:
        g = s.get(GatewayModel, gid)
        assert g.status == "running" and g.gateway_compute.ip_address == "203.0.113.7"
    assert calls[:2] == ["/api/healthcheck", "/api/config"]
    compute.create_gateway.assert_called_once()


def test_gateways_failed_if_creation_errors(db):
    from dstack_amd.server import background
    from dstack_amd.server.services import backends as backends_services

    with session_scope() as s:
        gid = _gateway(s)
    compute = mock.Mock()
    compute.create_gateway.side_effect = RuntimeError("quota exceeded")
    with mock.patch.object(backends_services, "get_project_backend", return_value=compute):
        background.process_submitted_gateways()
    with session_scope() as s:
        g = s.get(GatewayModel, gid)
        assert g.status == "failed" and "quota exceeded" in g.status_message


def test_gateways_failed_if_it_cannot_be_connected(db):
    from dstack_amd.server import background
    from dstack_amd.server.services import backends as backends_services
    from dstack_amd.server.services import gateways as gateways_services

    with session_scope() as s:
        gid = _gateway(s)
    compute = mock.Mock()
    compute.create_gateway.return_value = _gpd()
    down = mock.Mock(side_effect=ConnectionError("ssh: connect refused"))
    with mock.patch.object(backends_services, "get_project_backend", return_value=compute), \
            mock.patch.object(gateways_services, "_call", down):
        background.process_submitted_gateways()
        with session_scope() as s:
            assert s.get(GatewayModel, gid).status == "provisioning"  # still booting: retried
        later = get_current_datetime() + timedelta(seconds=gateways_services.GATEWAY_CONNECT_DEADLINE + 1)
        with mock.patch.object(gateways_services, "get_current_datetime", return_value=later):
            background.process_submitted_gateways()
    with session_scope() as s:
        g = s.get(GatewayModel, gid)
        assert g.status == "failed" and "Failed to connect to gateway" in g.status_message


# ---- process_instances --------------------------------------------------------------------------
def test_instances_terminate_calls_the_cloud(db):
    from dstack_amd.server.background.tasks import process_instances as pi

    with session_scope() as s:
        iid = _instance(s, status=InstanceStatus.TERMINATING)
    compute = mock.Mock()
    with mock.patch.object(pi.backends_services, "get_project_backend", return_value=compute), \
            session_scope() as s:
        pi._process_instance(s, iid)
    compute.terminate_instance.assert_called_once_with("i-1", "us-east-1", None)
    with session_scope() as s:
        inst = s.get(InstanceModel, iid)
        assert inst.status == "terminated" and inst.deleted and inst.finished_at is not None


def test_instances_terminate_not_retried_too_early(db):
    from dstack_amd.server.background.tasks import process_instances as pi

    with session_scope() as s:
        iid = _instance(s, status=InstanceStatus.TERMINATING)
    compute = mock.Mock()
    compute.terminate_instance.side_effect = RuntimeError("503")
    with mock.patch.object(pi.backends_services, "get_project_backend", return_value=compute):
        with session_scope() as s:
            pi._process_instance(s, iid)
        with session_scope() as s:  # a second pass within the minute: no new cloud call
            pi._process_instance(s, iid)
        assert compute.terminate_instance.call_count == 1
        with _at(timedelta(seconds=61)), session_scope() as s:
            pi._process_instance(s, iid)
        assert compute.terminate_instance.call_count == 2
    with session_scope() as s:
        assert s.get(InstanceModel, iid).status == "terminating"


def test_instances_idle_timeout_respects_fleet_policy(db):
    """``termination_policy: dont-destroy`` keeps an idle instance forever (reference: the second
    ``test_terminate_by_idle_timeout`` case)."""
    from dstack_amd.server.background.tasks import process_instances as pi

    with session_scope() as s:
        iid = _instance(s, status=InstanceStatus.IDLE, termination_policy="dont-destroy", termination_idle_time=60)
    with mock.patch.object(pi, "get_shim_client") as shim, _at(timedelta(hours=2)), session_scope() as s:
        shim.return_value.healthcheck.return_value = {"service": "dstack-shim"}
        shim.return_value.gpu_health.return_value = None
        pi._process_instance(s, iid)
    with session_scope() as s:
        assert s.get(InstanceModel, iid).status == "idle"


# ---- process_placement_groups -------------------------------------------------------------------
def test_placement_groups_of_deleted_fleets_deleted(db):
    from dstack_amd.server.background.tasks import process_placement_groups as ppg

    with session_scope() as s:
        project = s.query(ProjectModel).filter_by(name="main").one()
        fid = _fleet(s, "cluster")
        conf = {"backend": "aws", "region": "us-east-1", "placement_strategy": "cluster"}
        for name, deleted_fleet in (("pg-old", True), ("pg-live", False)):
            s.add(PlacementGroupModel(id=uuid.uuid4(), name=name, project_id=project.id, fleet_id=fid,
                                      configuration=json.dumps(conf), fleet_deleted=deleted_fleet))
    compute = mock.Mock()
    with mock.patch.object(ppg.backends_services, "get_project_backend", return_value=compute):
        ppg.process_placement_groups()
    assert [c.args[0].name for c in compute.delete_placement_group.call_args_list] == ["pg-old"]
    with session_scope() as s:
        state = {pg.name: pg.deleted for pg in s.query(PlacementGroupModel)}
    assert state == {"pg-old": True, "pg-live": False}


# ---- process_running_jobs -----------------------------------------------------------------------
def test_running_jobs_provisioning_job_unchanged_while_runner_not_alive(db):
    """A PROVISIONING job on a VM whose agent does not answer yet stays PROVISIONING (within the
    provisioning deadline), its submission is not touched."""
    from dstack_amd.server.background.tasks import process_running_jobs as prj

    with session_scope() as s:
        iid = _instance(s, status=InstanceStatus.BUSY)
        rid = _submit(s, {"type": "task", "commands": ["x"]})
        j = _job(s, rid)
        j.status = JobStatus.PROVISIONING.value
        j.instance_id = iid
        jpd = _jpd()
        jpd.dockerized = True
        j.job_provisioning_data = jpd.model_dump_json()
        jid = j.id
    shim = mock.Mock()
    shim.healthcheck.side_effect = ConnectionError("agent not up")
    shim.submit_task.side_effect = ConnectionError("agent not up")
    with mock.patch.object(prj, "get_shim_client", return_value=shim), session_scope() as s:
        prj._process_job(s, jid)
    with session_scope() as s:
        j = s.get(JobModel, jid)
        assert j.status == "provisioning" and j.termination_reason is None


# ---- process_submitted_jobs ---------------------------------------------------------------------
def test_submitted_job_fails_without_backends(db):
    """No backend configured at all (not even local): the job fails with no capacity."""
    from dstack_amd.server.background.tasks import process_submitted_jobs as psj
    from dstack_amd.server.services import backends as backends_services

    with session_scope() as s:
        rid = _submit(s, {"type": "task", "commands": ["x"]})
    with mock.patch.object(backends_services, "get_project_backends", return_value=[]), session_scope() as s:
        psj._process_job(s, _job(s, rid).id)
    with session_scope() as s:
        j = _job(s, rid)
        assert j.status in ("terminating", "failed")
        assert j.termination_reason == JobTerminationReason.FAILED_TO_START_DUE_TO_NO_CAPACITY.value


# ---- process_submitted_volumes ------------------------------------------------------------------
def _submitted_volume(s, backend="aws"):
    from dstack_amd.server.models import UserModel

    project = s.query(ProjectModel).filter_by(name="main").one()
    user = s.query(UserModel).filter_by(name="admin").one()
    v = VolumeModel(id=uuid.uuid4(), name="newvol", user_id=user.id, project_id=project.id, status="submitted",
                    configuration=json.dumps({"type": "volume", "name": "newvol", "backend": backend,
                                              "region": "us-east-1", "size": 100}),
                    created_at=get_current_datetime(), last_processed_at=get_current_datetime())
    s.add(v)
    s.flush()
    return v.id


def test_submitted_volume_fails_without_backend(db):
    from dstack_amd.server.background.tasks import process_volumes as pv

    with session_scope() as s:
        vid = _submitted_volume(s)
    with session_scope() as s:
        pv._process_volume(s, vid)
    with session_scope() as s:
        v = s.get(VolumeModel, vid)
        assert v.status == "failed" and v.status_message


def test_submitted_volume_provisioned(db):
    from dstack_amd.core.models.volumes import VolumeProvisioningData
    from dstack_amd.server.background.tasks import process_volumes as pv

    with session_scope() as s:
        vid = _submitted_volume(s)
    compute = mock.Mock()
    compute.create_volume.return_value = VolumeProvisioningData(backend=BackendType.AWS, volume_id="vol-123",
                                                                size_gb=100, availability_zone="us-east-1a")
    with mock.patch.object(pv.backends_services, "get_project_backend", return_value=compute), session_scope() as s:
        pv._process_volume(s, vid)
    with session_scope() as s:
        v = s.get(VolumeModel, vid)
        assert v.status == "active" and json.loads(v.volume_provisioning_data)["volume_id"] == "vol-123"


# ---- process_terminating_jobs on shared instances -----------------------------------------------
def _shared_instance_with_jobs(s, n_jobs=2, volume=False):
    """An 8-GPU instance split in 2 blocks, one running job per block (GPUs 0-3 and 4-7)."""
    from dstack_amd.core.models.common import NetworkMode
    from dstack_amd.core.models.runs import JobRuntimeData

    iid = _instance(s, status=InstanceStatus.BUSY)
    inst = s.get(InstanceModel, iid)
    inst.total_blocks = 2
    inst.busy_blocks = n_jobs
    inst.busy_gpus = ",".join(str(i) for i in range(4 * n_jobs))
    offer = json.loads(inst.offer)
    offer["total_blocks"] = 2
    offer["blocks"] = 1
    jobs = []
    for k in range(n_jobs):
        rid = _submit(s, {"type": "task", "commands": ["x"]}, name=f"shared-{k}")
        j = _job(s, rid)
        j.status = JobStatus.TERMINATING.value if k == 0 else JobStatus.RUNNING.value
        j.termination_reason = JobTerminationReason.TERMINATED_BY_USER.value if k == 0 else None
        j.instance_id = iid
        j.job_provisioning_data = _jpd().model_dump_json()
        from dstack_amd.core.models.instances import InstanceOfferWithAvailability

        j.job_runtime_data = JobRuntimeData(network_mode=NetworkMode.BRIDGE, gpu=4,
                                            offer=InstanceOfferWithAvailability.model_validate(offer),
                                            gpu_indices=list(range(4 * k, 4 * k + 4)),
                                            volume_names=["shared-data"] if volume else None).model_dump_json()
        jobs.append(j.id)
    return iid, jobs


def test_terminating_job_on_shared_instance_frees_only_its_block(db):
    from dstack_amd.server.background.tasks import process_terminating_jobs as ptj

    with session_scope() as s:
        iid, (jid, other) = _shared_instance_with_jobs(s)
    shim = mock.Mock()
    with mock.patch.object(ptj, "get_shim_client", return_value=shim), session_scope() as s:
        ptj._process_job(s, jid)
    shim.terminate_task.assert_called_once()
    assert shim.terminate_task.call_args[0][0] == str(jid)
    with session_scope() as s:
        j = s.get(JobModel, jid)
        inst = s.get(InstanceModel, iid)
        assert j.status == "terminated" and j.instance_id is None and j.used_instance_id == iid
        assert inst.busy_blocks == 1 and inst.busy_gpus == "4,5,6,7" and inst.status == "busy"


def test_terminating_job_on_shared_instance_keeps_volume_used_by_the_other_job(db):
    from dstack_amd.server.background.tasks import process_terminating_jobs as ptj
    from dstack_amd.server.services import backends as backends_services
    from tests.test_volumes_jobs import _volume

    with session_scope() as s:
        vid = _volume(s, name="shared-data")
        iid, (jid, other) = _shared_instance_with_jobs(s, volume=True)
        s.execute(volumes_attachments.insert().values(volume_id=vid, instance_id=iid))
    compute = mock.Mock()
    with mock.patch.object(backends_services, "get_project_backend", return_value=compute), \
            mock.patch.object(ptj, "get_shim_client", return_value=mock.Mock()), session_scope() as s:
        ptj._process_job(s, jid)
    compute.detach_volume.assert_not_called()  # the other job on the host still mounts it
    with session_scope() as s:
        assert s.get(JobModel, jid).status == "terminated"
        assert list(s.execute(select(volumes_attachments.c.instance_id)
                              .where(volumes_attachments.c.volume_id == vid)).scalars()) == [iid]
