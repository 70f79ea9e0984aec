"""Delete placement groups of deleted fleets (reference:
``S/background/tasks/process_placement_groups.py:20-96``)."""

from __future__ import annotations

import logging

from sqlalchemy import select

from dstack_amd.core.models.placement import PlacementGroup, PlacementGroupConfiguration
from dstack_amd.server.db import session_scope
from dstack_amd.server.models import PlacementGroupModel
from dstack_amd.server.services import backends as backends_services
from dstack_amd.utils.common import get_current_datetime

logger = logging.getLogger(__name__)


def process_placement_groups() -> bool:
    with session_scope() as s:
        rows = list(s.execute(select(PlacementGroupModel).where(PlacementGroupModel.fleet_deleted == True,  # noqa
                                                                PlacementGroupModel.deleted == False)).scalars())  # noqa
        for pg in rows:
            conf = PlacementGroupConfiguration.model_validate_json(pg.configuration)
            try:
                compute = backends_services.get_project_backend(s, pg.project, conf.backend)
                compute.delete_placement_group(PlacementGroup(name=pg.name, project_name=pg.project.name,
                                                              configuration=conf))
            except NotImplementedError:
                pass
            except Exception as e:  # noqa: BLE001
                logger.warning("placement group %s: delete failed: %s", pg.name, e)
                continue
            pg.deleted = True
            pg.deleted_at = get_current_datetime()
    return False
