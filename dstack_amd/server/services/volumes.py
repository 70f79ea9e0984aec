"""Volumes (reference: ``S/services/volumes.py:38-355``): CRUD, job mount resolution and attach
checks.  MI355X: new volumes without ``size`` get a size sized from the 288 GB HBM per GPU of the
project's largest fleet host (``recommended_volume_size_gb``)."""

from __future__ import annotations

import uuid
from typing import List, Optional

from sqlalchemy import select
from sqlalchemy.orm import Session

from dstack_amd.core.errors import ResourceExistsError, ResourceNotExistsError, ServerClientError
from dstack_amd.core.models.backends import BACKENDS_WITH_VOLUMES_SUPPORT
from dstack_amd.core.models.volumes import (
    Volume,
    VolumeAttachmentData,
    VolumeConfiguration,
    VolumePlan,
    VolumeProvisioningData,
    VolumeSpec,
    VolumeStatus,
    recommended_volume_size_gb,
)
from dstack_amd.server.background import scheduler
from dstack_amd.server.models import ProjectModel, UserModel, VolumeModel
from dstack_amd.utils.common import generate_name, get_current_datetime


def volume_model_to_volume(v: VolumeModel) -> Volume:
    conf = VolumeConfiguration.model_validate_json(v.configuration)
    vpd = VolumeProvisioningData.model_validate_json(v.volume_provisioning_data) if v.volume_provisioning_data else None
    vad = VolumeAttachmentData.model_validate_json(v.volume_attachment_data) if v.volume_attachment_data else None
    return Volume(id=v.id, name=v.name, user=v.user.name if v.user else "", project_name=v.project.name,
                  configuration=conf, external=conf.volume_id is not None, created_at=v.created_at,
                  status=VolumeStatus(v.status), status_message=v.status_message, deleted=v.deleted,
                  volume_id=vpd.volume_id if vpd else None, provisioning_data=vpd, attachment_data=vad)


def list_project_volumes(s: Session, project: ProjectModel) -> List[VolumeModel]:
    return list(s.execute(select(VolumeModel).where(VolumeModel.project_id == project.id,
                                                    VolumeModel.deleted == False)  # noqa: E712
                          .order_by(VolumeModel.created_at)).scalars())


def get_volume_by_name(s: Session, project: ProjectModel, name: str) -> Optional[VolumeModel]:
    return s.execute(select(VolumeModel).where(VolumeModel.project_id == project.id, VolumeModel.name == name,
                                               VolumeModel.deleted == False)).scalar_one_or_none()  # noqa: E712


def get_plan(s: Session, project: ProjectModel, user: UserModel, spec: VolumeSpec) -> VolumePlan:
    cur = get_volume_by_name(s, project, spec.configuration.name) if spec.configuration.name else None
    return VolumePlan(project_name=project.name, user=user.name, spec=spec,
                      current_resource=volume_model_to_volume(cur) if cur else None)


def create_volume(s: Session, project: ProjectModel, user: UserModel, conf: VolumeConfiguration) -> Volume:
    if conf.backend not in BACKENDS_WITH_VOLUMES_SUPPORT:
        raise ServerClientError(f"Backend {conf.backend.value} does not support volumes")
    if conf.volume_id is None and conf.size is None:
        conf.size = recommended_volume_size_gb(8)
    if conf.name is None:
        conf.name = generate_name()
    if get_volume_by_name(s, project, conf.name) is not None:
        raise ResourceExistsError(f"Volume {conf.name} exists")
    v = VolumeModel(id=uuid.uuid4(), name=conf.name, user_id=user.id, project_id=project.id,
                    status=VolumeStatus.SUBMITTED.value, configuration=conf.model_dump_json(),
                    created_at=get_current_datetime(), last_processed_at=get_current_datetime())
    s.add(v)
    s.flush()
    s.refresh(v)
    scheduler.wake(scheduler.VOLUMES)
    return volume_model_to_volume(v)


def delete_volumes(s: Session, project: ProjectModel, names: List[str]):
    """Held in the volumes lockset and committed inside, so a job attaching a volume concurrently
    (``jobs.volumes.attach_job_volumes``, same lock) cannot slip past the attachment check."""
    from dstack_amd.server.services.locking import lockset

    vols = []
    for n in names:
        v = get_volume_by_name(s, project, n)
        if v is None:
            raise ResourceNotExistsError(f"Volume {n} not found")
        vols.append(v)
    with lockset("volumes").hold([v.id for v in vols], timeout=60.0):
        for v in vols:
            s.refresh(v, with_for_update=True)
        _delete_volumes_locked(s, project, vols)
        s.commit()


def _delete_volumes_locked(s: Session, project: ProjectModel, vols):
    # check every volume before deleting any in the cloud: a rejected volume later in the list
    # must not leave an earlier one deleted in the cloud but ACTIVE in the (rolled back) database
    for v in vols:
        if v.instances:
            raise ServerClientError(f"Volume {v.name} is attached to an instance")
    for v in vols:
        conf = VolumeConfiguration.model_validate_json(v.configuration)
        if conf.volume_id is None and v.volume_provisioning_data:
            from dstack_amd.server.services import backends as backends_services

            try:
                backends_services.get_project_backend(s, project, conf.backend).delete_volume(volume_model_to_volume(v))
            except NotImplementedError:
                pass
        v.deleted = True
        v.deleted_at = get_current_datetime()
