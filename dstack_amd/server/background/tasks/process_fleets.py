"""Auto-delete fleets whose instances are all gone (reference:
``S/background/tasks/process_fleets.py:19-83``); placement groups of deleted fleets are marked for
deletion."""

from __future__ import annotations

import json

from sqlalchemy import select
from sqlalchemy.orm import Session

from dstack_amd.core.models.fleets import FleetStatus
from dstack_amd.core.models.instances import InstanceStatus
from dstack_amd.core.models.runs import RunStatus
from dstack_amd.server.background.common import claim_and_process
from dstack_amd.server.models import FleetModel, PlacementGroupModel, RunModel
from dstack_amd.utils.common import get_current_datetime


def process_fleets(batch: int = 10) -> bool:
    def select_ids(s: Session):
        return s.execute(select(FleetModel.id).where(FleetModel.deleted == False)  # noqa: E712
                         .order_by(FleetModel.last_processed_at).limit(batch * 4)).scalars()

    return claim_and_process("fleets", select_ids, _process_fleet, batch)


def _process_fleet(s: Session, fleet_id):
    f = s.get(FleetModel, fleet_id)
    if f is None or f.deleted:
        return
    f.last_processed_at = get_current_datetime()
    live = [i for i in f.instances if i.status != InstanceStatus.TERMINATED.value]
    active_runs = s.execute(select(RunModel).where(RunModel.fleet_id == f.id, RunModel.status.notin_(
        [x.value for x in RunStatus.finished_statuses()]))).scalars().first()
    spec = json.loads(f.spec)
    autocreated = spec.get("autocreated", False)
    terminating = f.status == FleetStatus.TERMINATING.value
    nodes_min = ((spec.get("configuration") or {}).get("nodes") or {}).get("min")
    empty_allowed = nodes_min == 0
    if live or active_runs is not None:
        return
    if not (autocreated or terminating) or (empty_allowed and not terminating):
        return
    f.status = FleetStatus.TERMINATED.value
    f.deleted = True
    f.deleted_at = get_current_datetime()
    for pg in s.execute(select(PlacementGroupModel).where(PlacementGroupModel.fleet_id == f.id)).scalars():
        pg.fleet_deleted = True
