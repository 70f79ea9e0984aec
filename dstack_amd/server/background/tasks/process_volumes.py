"""SUBMITTED volumes -> ACTIVE via the backend's create/register (reference:
``S/background/tasks/process_volumes.py:18-112``)."""

from __future__ import annotations

import logging

from sqlalchemy import select
from sqlalchemy.orm import Session

from dstack_amd.core.models.volumes import VolumeConfiguration, VolumeStatus
from dstack_amd.server.background.common import claim_and_process
from dstack_amd.server.models import VolumeModel
from dstack_amd.server.services import backends as backends_services
from dstack_amd.server.services import volumes as volumes_services
from dstack_amd.utils.common import get_current_datetime

logger = logging.getLogger(__name__)


def process_submitted_volumes(batch: int = 5) -> bool:
    def select_ids(s: Session):
        return s.execute(select(VolumeModel.id).where(VolumeModel.status == VolumeStatus.SUBMITTED.value,
                                                      VolumeModel.deleted == False)  # noqa: E712
                         .order_by(VolumeModel.last_processed_at).limit(batch * 4)).scalars()

    return claim_and_process("volumes", select_ids, _process_volume, batch)


def _process_volume(s: Session, vid):
    v = s.get(VolumeModel, vid)
    if v is None or v.status != VolumeStatus.SUBMITTED.value:
        return
    v.last_processed_at = get_current_datetime()
    conf = VolumeConfiguration.model_validate_json(v.configuration)
    try:
        compute = backends_services.get_project_backend(s, v.project, conf.backend)
        vol = volumes_services.volume_model_to_volume(v)
        vpd = compute.register_volume(vol) if conf.volume_id else compute.create_volume(vol)
    except Exception as e:  # noqa: BLE001
        v.status = VolumeStatus.FAILED.value
        v.status_message = str(e)[:1000]
        return
    v.volume_provisioning_data = vpd.model_dump_json()
    v.status = VolumeStatus.ACTIVE.value
