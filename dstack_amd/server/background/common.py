"""Shared claim/process helper for reconcilers: select the oldest rows, claim them in a lockset,
process each in its own session (the pattern of ``process_running_jobs.py:68-93``)."""

from __future__ import annotations

import logging
from typing import Callable, Iterable, List

from sqlalchemy.orm import Session

from dstack_amd.server.db import session_scope
from dstack_amd.server.services.locking import claim_row, lockset

logger = logging.getLogger(__name__)


def _model_for(namespace: str):
    from dstack_amd.server import models

    return {
        "jobs": models.JobModel, "runs": models.RunModel, "instances": models.InstanceModel,
        "fleets": models.FleetModel, "gateways": models.GatewayModel, "volumes": models.VolumeModel,
        "placement_groups": models.PlacementGroupModel,
    }.get(namespace)


def claim_and_process(namespace: str, select_ids: Callable[[Session], Iterable],
                      process_one: Callable[[Session, object], None], batch: int = 5) -> bool:
    """Returns True when a full batch was processed (the scheduler re-runs immediately).

    Each row is processed in its own transaction; on Postgres the row is first claimed with
    ``FOR UPDATE SKIP LOCKED`` so that concurrent server replicas never process it twice."""
    model = _model_for(namespace)
    ls = lockset(namespace)
    with session_scope() as s:
        candidates = list(select_ids(s))
    ids: List = []
    for c in candidates:
        if len(ids) >= batch:
            break
        ids += ls.try_add_many([c])
    done: List = []
    try:
        for item_id in ids:
            try:
                with session_scope() as s:
                    if model is not None and not claim_row(s, model, item_id):
                        continue  # another server replica holds it
                    process_one(s, item_id)
            except Exception:  # noqa: BLE001
                logger.exception("%s: processing %s failed", namespace, item_id)
            finally:
                # released per item once its transaction ended: a request waiting on this row
                # (stop/delete under Lockset.hold) does not wait for the rest of the batch
                ls.remove_many([item_id])
                done.append(item_id)
    finally:
        ls.remove_many([i for i in ids if i not in done])
    return len(ids) >= batch
