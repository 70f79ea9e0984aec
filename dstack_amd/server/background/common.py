"""Shared claim/process helper for reconcilers: select the oldest rows, claim them in a lockset,
process each in its own session (the pattern of ``process_running_jobs.py:68-93``)."""

from __future__ import annotations

import logging
from typing import Callable, Iterable, List

from sqlalchemy.orm import Session

from dstack_amd.server.db import session_scope
from dstack_amd.server.services.locking import lockset

logger = logging.getLogger(__name__)


def claim_and_process(namespace: str, select_ids: Callable[[Session], Iterable],
                      process_one: Callable[[Session, object], None], batch: int = 5) -> bool:
    """Returns True when a full batch was processed (the scheduler re-runs immediately)."""
    ls = lockset(namespace)
    with session_scope() as s:
        candidates = list(select_ids(s))
    ids: List = []
    for c in candidates:
        if len(ids) >= batch:
            break
        ids += ls.try_add_many([c])
    try:
        for item_id in ids:
            try:
                with session_scope() as s:
                    process_one(s, item_id)
            except Exception:  # noqa: BLE001
                logger.exception("%s: processing %s failed", namespace, item_id)
    finally:
        ls.remove_many(ids)
    return len(ids) >= batch
