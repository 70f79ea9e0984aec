"""Network volumes through the job lifecycle (reference:
``src/tests/_internal/server/background/tasks/test_process_submitted_jobs.py`` volume cases and
``test_process_terminating_jobs.py`` detach cases): placement is pinned to the volume's
backend/region, missing or inactive volumes fail the job with ``volume_error``, the volume is
attached before the shim submit and described in the shim body, and detached (soft, then forced
after ``stop_duration``) on termination."""

import json
import uuid
from datetime import timedelta
from unittest import mock

from sqlalchemy import select

from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.runs import JobStatus, JobTerminationReason
from dstack_amd.core.models.volumes import VolumeAttachmentData, VolumeStatus
from dstack_amd.server.db import session_scope
from dstack_amd.server.models import InstanceModel, JobModel, ProjectModel, UserModel, VolumeModel, volumes_attachments
from dstack_amd.utils.common import get_current_datetime

from tests.test_reconcilers import _instance, _job, _jpd, _submit


def _volume(s, name="data", region="us-east-1", status=VolumeStatus.ACTIVE, external=False):
    project = s.query(ProjectModel).filter_by(name="main").one()
    user = s.query(UserModel).filter_by(name="admin").one()
    conf = {"type": "volume", "name": name, "backend": "aws", "region": region, "size": 100}
    if external:
        conf["volume_id"] = "vol-ext"
    v = VolumeModel(id=uuid.uuid4(), name=name, user_id=user.id, project_id=project.id, status=status.value,
                    configuration=json.dumps(conf),
                    volume_provisioning_data='{"volume_id": "vol-0abc", "size_gb": 100}',
                    created_at=get_current_datetime(), last_processed_at=get_current_datetime())
    s.add(v)
    s.flush()
    return v.id


TASK = {"type": "task", "commands": ["ls /data"], "volumes": ["data:/data"]}


def test_job_placed_only_on_instance_in_volume_region(db):
    from dstack_amd.server.background.tasks import process_submitted_jobs as psj

    with session_scope() as s:
        _volume(s, region="us-east-1")
        iid = _instance(s)  # aws / us-east-1
        rid = _submit(s, TASK)
    with session_scope() as s:
        psj._process_job(s, _job(s, rid).id)
    with session_scope() as s:
        j = _job(s, rid)
        assert j.status == "provisioning" and j.instance_id == iid


def test_volume_in_other_region_excludes_pool_instance_and_offers(db):
    from dstack_amd.core.models.instances import InstanceAvailability, InstanceOfferWithAvailability
    from dstack_amd.server.background.tasks import process_submitted_jobs as psj

    from tests.test_reconcilers import _itype

    with session_scope() as s:
        _volume(s, region="eu-west-1")
        _instance(s)  # us-east-1: must not be reused
        rid = _submit(s, TASK)
    offer = InstanceOfferWithAvailability(backend=BackendType.AWS, instance=_itype(), region="us-east-1", price=1.0,
                                          availability=InstanceAvailability.AVAILABLE)
    compute = mock.Mock()
    with mock.patch.object(psj.offers_services, "get_offers_by_requirements", return_value=[(compute, offer)]), \
            session_scope() as s:
        psj._process_job(s, _job(s, rid).id)
    compute.run_job.assert_not_called()
    with session_scope() as s:
        j = _job(s, rid)
        assert j.termination_reason == JobTerminationReason.FAILED_TO_START_DUE_TO_NO_CAPACITY.value


def test_missing_or_inactive_volume_fails_with_volume_error(db):
    from dstack_amd.server.background.tasks import process_submitted_jobs as psj

    with session_scope() as s:
        rid = _submit(s, TASK, name="nov")
    with session_scope() as s:
        psj._process_job(s, _job(s, rid).id)
    with session_scope() as s:
        assert _job(s, rid).termination_reason == JobTerminationReason.VOLUME_ERROR.value
        _volume(s, status=VolumeStatus.PROVISIONING)
        rid2 = _submit(s, TASK, name="inactive")
    with session_scope() as s:
        psj._process_job(s, _job(s, rid2).id)
    with session_scope() as s:
        j = _job(s, rid2)
        assert j.termination_reason == JobTerminationReason.VOLUME_ERROR.value
        assert "not active" in (j.termination_reason_message or "")


def _provisioning_job(s, rid, iid):
    from dstack_amd.core.models.common import NetworkMode
    from dstack_amd.core.models.runs import JobRuntimeData

    j = _job(s, rid)
    j.status = JobStatus.PROVISIONING.value
    j.instance_id = iid
    j.job_provisioning_data = _jpd().model_dump_json()
    j.job_runtime_data = JobRuntimeData(network_mode=NetworkMode.HOST).model_dump_json()
    s.get(InstanceModel, iid).status = "busy"
    return j.id


def test_volume_attached_before_shim_submit_and_detached_on_termination(db):
    from dstack_amd.server.background.tasks import process_running_jobs as prj
    from dstack_amd.server.background.tasks import process_terminating_jobs as ptj
    from dstack_amd.server.services import backends as backends_services
    from dstack_amd.server.services import jobs as jobs_services

    with session_scope() as s:
        vid = _volume(s)
        iid = _instance(s)
        rid = _submit(s, TASK)
        jid = _provisioning_job(s, rid, iid)
    compute = mock.Mock()
    compute.attach_volume.return_value = VolumeAttachmentData(device_name="/dev/sdf")
    compute.is_volume_detached.return_value = False
    shim = mock.Mock()
    with mock.patch.object(backends_services, "get_project_backend", return_value=compute), \
            mock.patch.object(prj, "get_shim_client", return_value=shim):
        with session_scope() as s:
            j = s.get(JobModel, jid)
            prj._process_provisioning(s, j.run, j)
        compute.attach_volume.assert_called_once()
        assert compute.attach_volume.call_args[0][1] == "i-1"  # the cloud instance id
        body = shim.submit_task.call_args[0][0]
        assert body["volumes"] == [{"backend": "aws", "name": "data", "volume_id": "vol-0abc",
                                    "device_name": "/dev/sdf", "init_fs": True}]
        assert body["volume_mounts"] == [{"name": "data", "path": "/data"}]
        with session_scope() as s:
            j = s.get(JobModel, jid)
            assert j.status == "pulling" and jobs_services.job_jrd(j).volume_names == ["data"]
            assert list(s.execute(select(volumes_attachments.c.instance_id)
                                  .where(volumes_attachments.c.volume_id == vid)).scalars()) == [iid]
            jobs_services.terminate_job(j, JobTerminationReason.TERMINATED_BY_USER, delay=False)
        # soft detach still in progress: the job stays terminating, but the instance is released
        # already -- a stuck volume never holds the host (reference test_force_detaches_job_volumes)
        with mock.patch.object(ptj, "get_shim_client", return_value=shim), session_scope() as s:
            ptj._process_job(s, jid)
        with session_scope() as s:
            j = s.get(JobModel, jid)
            assert j.status == "terminating" and j.instance_id is None and j.used_instance_id == iid
            assert j.volumes_detached_at is not None
            assert s.get(InstanceModel, iid).busy_blocks == 0
            assert list(s.execute(select(volumes_attachments.c.instance_id)
                                  .where(volumes_attachments.c.volume_id == vid)).scalars()) == [iid]
        assert compute.detach_volume.call_args.kwargs.get("force") is False
        # past stop_duration + grace: forced detach, then the job finishes
        compute.is_volume_detached.return_value = True
        later = get_current_datetime() + timedelta(minutes=10)
        with mock.patch("dstack_amd.server.services.jobs.volumes.get_current_datetime", return_value=later), \
                mock.patch.object(ptj, "get_shim_client", return_value=shim), session_scope() as s:
            ptj._process_job(s, jid)
        assert compute.detach_volume.call_args.kwargs.get("force") is True
    with session_scope() as s:
        j = s.get(JobModel, jid)
        assert j.status == "terminated" and j.volumes_detached_at is not None
        assert not list(s.execute(select(volumes_attachments).where(volumes_attachments.c.volume_id == vid)))
        assert s.get(VolumeModel, vid).volume_attachment_data is None


def test_external_volume_not_formatted_and_attach_failure_is_volume_error(db):
    from dstack_amd.core.errors import ComputeError
    from dstack_amd.server.background.tasks import process_running_jobs as prj
    from dstack_amd.server.services import backends as backends_services

    with session_scope() as s:
        _volume(s, external=True)
        iid = _instance(s)
        rid = _submit(s, TASK)
        jid = _provisioning_job(s, rid, iid)
    compute = mock.Mock()
    compute.attach_volume.side_effect = ComputeError("VolumeInUse")
    with mock.patch.object(backends_services, "get_project_backend", return_value=compute), \
            mock.patch.object(prj, "get_shim_client", return_value=mock.Mock()), session_scope() as s:
        j = s.get(JobModel, jid)
        prj._process_provisioning(s, j.run, j)
    with session_scope() as s:
        j = s.get(JobModel, jid)
        assert j.termination_reason == JobTerminationReason.VOLUME_ERROR.value
    from dstack_amd.server.services.jobs.volumes import shim_volume_specs

    with session_scope() as s:
        assert shim_volume_specs(s, s.get(JobModel, jid), ["data"])[0]["init_fs"] is False



def test_volume_attach_waits_for_a_concurrent_delete(db):
    """A delete holds the volume (volumes lockset) until it commits: an attach arriving while the
    cloud delete is in progress waits, then re-reads the volume and sees it deleted (the attach
    path then refuses it) instead of attaching a volume that is being deleted."""
    import threading
    import time

    from dstack_amd.server.services import backends as backends_services
    from dstack_amd.server.services import volumes as volumes_services
    from dstack_amd.server.services.jobs.volumes import _hold_volume

    with session_scope() as s:
        vid = _volume(s)
    deleting = threading.Event()
    seen = {}

    def slow_delete(_vol):
        deleting.set()
        time.sleep(0.3)

    def attach():
        assert deleting.wait(5)
        with session_scope() as s:
            v = s.get(VolumeModel, vid)
            _hold_volume(s, v)
            seen["deleted"] = v.deleted

    compute = mock.Mock()
    compute.delete_volume.side_effect = slow_delete
    t = threading.Thread(target=attach)
    t.start()
    with mock.patch.object(backends_services, "get_project_backend", return_value=compute), session_scope() as s:
        volumes_services.delete_volumes(s, s.query(ProjectModel).filter_by(name="main").one(), ["data"])
    t.join(5)
    assert seen == {"deleted": True}


def test_volume_busy_retries_instead_of_failing_the_job(db):
    """Another job's attach transaction still holds the volume (e.g. while its shim call is slow):
    this job is retried on a later pass, not terminated with VOLUME_ERROR."""
    from dstack_amd.server.background.tasks import process_running_jobs as prj
    from dstack_amd.server.services import backends as backends_services
    from dstack_amd.server.services.locking import lockset

    with session_scope() as s:
        vid = _volume(s)
        iid = _instance(s)
        rid = _submit(s, TASK)
        jid = _provisioning_job(s, rid, iid)
    compute = mock.Mock()
    compute.attach_volume.return_value = VolumeAttachmentData(device_name="/dev/sdf")
    shim = mock.Mock()
    lockset("volumes").add_all_or_nothing([vid])
    try:
        with mock.patch.object(backends_services, "get_project_backend", return_value=compute), \
                mock.patch.object(prj, "get_shim_client", return_value=shim), session_scope() as s:
            j = s.get(JobModel, jid)
            prj._process_provisioning(s, j.run, j)
    finally:
        lockset("volumes").remove_many([vid])
    with session_scope() as s:
        j = s.get(JobModel, jid)
        assert j.status == "provisioning" and j.termination_reason is None
    shim.submit_task.assert_not_called()
    with mock.patch.object(backends_services, "get_project_backend", return_value=compute), \
            mock.patch.object(prj, "get_shim_client", return_value=shim), session_scope() as s:
        j = s.get(JobModel, jid)
        prj._process_provisioning(s, j.run, j)
    with session_scope() as s:
        assert s.get(JobModel, jid).status == "pulling"
    shim.submit_task.assert_called_once()


def test_delete_volumes_checks_all_before_any_cloud_delete(db):
    """Deleting [v1, v2] with v2 attached: nothing is deleted in the cloud (v1 would otherwise be
    gone in the cloud yet ACTIVE in the rolled-back database)."""
    import pytest

    from dstack_amd.core.errors import ServerClientError
    from dstack_amd.server.services import backends as backends_services
    from dstack_amd.server.services import volumes as volumes_services

    with session_scope() as s:
        _volume(s, name="v1")
        v2 = _volume(s, name="v2")
        iid = _instance(s)
        s.execute(volumes_attachments.insert().values(volume_id=v2, instance_id=iid, attachment_data="{}"))
    compute = mock.Mock()
    with mock.patch.object(backends_services, "get_project_backend", return_value=compute), session_scope() as s:
        with pytest.raises(ServerClientError, match="v2 is attached"):
            volumes_services.delete_volumes(s, s.query(ProjectModel).filter_by(name="main").one(), ["v1", "v2"])
    compute.delete_volume.assert_not_called()
    with session_scope() as s:
        assert not s.query(VolumeModel).filter_by(name="v1").one().deleted
