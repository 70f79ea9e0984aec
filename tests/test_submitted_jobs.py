"""``process_submitted_jobs`` provisioning decisions against fake backends (reference:
``src/tests/_internal/server/background/tasks/test_process_submitted_jobs.py``): privileged runs and
required instance mounts only go to VM backends, an optional instance mount does not restrict the
offers, and a run bound to a fleet grows that fleet only while it is a cloud fleet below
``nodes.max`` (SSH fleets have exactly their hosts)."""

from __future__ import annotations

from typing import List
from unittest import mock

from dstack_amd.core.backends.base import Compute
from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.instances import (
    InstanceAvailability,
    InstanceOfferWithAvailability,
    InstanceStatus,
    InstanceType,
    Resources,
)
from dstack_amd.core.models.runs import JobProvisioningData, JobStatus, JobTerminationReason, RunSpec
from dstack_amd.server.background.tasks import process_submitted_jobs as psj
from dstack_amd.server.db import session_scope
from dstack_amd.server.models import FleetModel, InstanceModel, JobModel, ProjectModel, UserModel
from dstack_amd.server.services import backends as backends_services
from dstack_amd.server.services import fleets as fleets_services
from dstack_amd.server.services import runs as runs_services


class FakeCompute(Compute):
    def __init__(self, backend: BackendType):
        self.backend = backend
        self.run_job_calls: List[str] = []

    def get_offers(self, requirements=None):
        it = InstanceType(name="instance", resources=Resources(cpus=4, memory_mib=8192, spot=False, gpus=[]))
        return [InstanceOfferWithAvailability(backend=self.backend, instance=it, region="us", price=1.0,
                                              availability=InstanceAvailability.AVAILABLE)]

    def get_offers_cached(self, requirements=None):
        return self.get_offers(requirements)

    def run_job(self, run, job, offer, project_ssh_public_key, project_ssh_private_key, volumes):
        self.run_job_calls.append(offer.backend.value)
        return JobProvisioningData(backend=offer.backend, instance_type=offer.instance, instance_id="i-1",
                                   hostname="1.1.1.1", internal_ip=None, region=offer.region, price=offer.price,
                                   username="ubuntu", ssh_port=22, dockerized=True)

    def terminate_instance(self, instance_id, region, backend_data=None):
        pass


def _submit(conf: dict, name="run1"):
    with session_scope() as s:
        project = s.query(ProjectModel).filter_by(name="main").one()
        user = s.query(UserModel).filter_by(name="admin").one()
        spec = RunSpec.model_validate({"run_name": name, "repo_id": "virt", "repo_data": {"repo_type": "virtual"},
                                       "configuration": {"type": "task", "commands": ["true"], **conf}})
        run_id = runs_services.submit_run(s, project, user, spec).id
        return run_id, [j.id for j in s.query(JobModel).filter_by(run_id=run_id)]


def _process(job_id, backends):
    with mock.patch.object(backends_services, "get_project_backends", return_value=backends):
        with session_scope() as s:
            psj._process_job(s, job_id)
    with session_scope() as s:
        j = s.get(JobModel, job_id)
        return j.status, j.termination_reason, j.instance


def _no_capacity(result):
    status, reason, inst = result
    return (status == JobStatus.TERMINATING.value and inst is None
            and reason == JobTerminationReason.FAILED_TO_START_DUE_TO_NO_CAPACITY.value)


def test_privileged_run_skips_container_backends(db):
    runpod = FakeCompute(BackendType.RUNPOD)
    _, (jid,) = _submit({"privileged": True})
    assert _no_capacity(_process(jid, [(BackendType.RUNPOD, runpod)]))
    assert runpod.run_job_calls == []
    aws = FakeCompute(BackendType.AWS)
    _, (jid,) = _submit({"privileged": True}, name="run2")
    status, _, _ = _process(jid, [(BackendType.RUNPOD, runpod), (BackendType.AWS, aws)])
    assert status == JobStatus.PROVISIONING.value and aws.run_job_calls == ["aws"] and runpod.run_job_calls == []


def test_required_instance_mount_needs_vm_backend(db):
    runpod = FakeCompute(BackendType.RUNPOD)
    _, (jid,) = _submit({"volumes": ["/root/.cache:/cache"]})
    assert _no_capacity(_process(jid, [(BackendType.RUNPOD, runpod)]))
    assert runpod.run_job_calls == []


def test_optional_instance_mount_does_not_restrict_offers(db):
    runpod = FakeCompute(BackendType.RUNPOD)
    _, (jid,) = _submit({"volumes": [{"instance_path": "/root/.cache", "path": "/cache", "optional": True}]})
    status, _, inst = _process(jid, [(BackendType.RUNPOD, runpod)])
    assert status == JobStatus.PROVISIONING.value and runpod.run_job_calls == ["runpod"]
    assert inst is not None and inst.backend == "runpod"


def _bind_run_to_fleet(run_id, conf: dict) -> str:
    from dstack_amd.core.models.fleets import FleetSpec

    with session_scope() as s:
        project = s.query(ProjectModel).filter_by(name="main").one()
        user = s.query(UserModel).filter_by(name="admin").one()
        spec = FleetSpec.model_validate({"configuration": {"type": "fleet", **conf}, "profile": {"name": "default"}})
        fleet = fleets_services.create_fleet(s, project, user, spec)
        for i in fleet.instances:  # the fleet's existing nodes are all busy
            i.status = InstanceStatus.BUSY.value
        from dstack_amd.server.models import RunModel

        s.get(RunModel, run_id).fleet_id = fleet.id
        return fleet.id


def test_new_instance_created_in_cloud_fleet_below_max(db):
    aws = FakeCompute(BackendType.AWS)
    run_id, (jid,) = _submit({})
    fid = _bind_run_to_fleet(run_id, {"name": "cloud", "nodes": "1..2"})
    status, _, _ = _process(jid, [(BackendType.AWS, aws)])
    assert status == JobStatus.PROVISIONING.value
    with session_scope() as s:
        j = s.get(JobModel, jid)
        assert j.instance.fleet_id == fid and j.instance.instance_num == 1
        assert s.query(FleetModel).count() == 1  # no autocreated fleet


def test_fleet_at_max_or_ssh_fleet_does_not_grow(db):
    aws = FakeCompute(BackendType.AWS)
    run_id, (jid,) = _submit({})
    _bind_run_to_fleet(run_id, {"name": "full", "nodes": 1})
    assert _no_capacity(_process(jid, [(BackendType.AWS, aws)]))
    key = {"public": "ssh-ed25519 AAAA", "private": "-----BEGIN OPENSSH PRIVATE KEY-----\nx\n"
                                                   "-----END OPENSSH PRIVATE KEY-----\n"}
    run_id, (jid,) = _submit({}, name="run2")
    _bind_run_to_fleet(run_id, {"name": "onprem", "ssh_config": {"user": "u", "ssh_key": key, "hosts": ["10.0.0.9"]}})
    assert _no_capacity(_process(jid, [(BackendType.AWS, aws)]))
    assert aws.run_job_calls == []
    with session_scope() as s:
        assert s.query(InstanceModel).filter(InstanceModel.backend == "aws").count() == 0
