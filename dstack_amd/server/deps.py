"""FastAPI dependencies (reference: ``S/deps.py``)."""

from __future__ import annotations

from typing import Iterator

from sqlalchemy.orm import Session

from dstack_amd.server.db import get_db


def get_session() -> Iterator[Session]:
    """One session per request, committed when the endpoint returns.  Routes declare it with
    ``Depends(get_session, scope="function")`` so the commit runs BEFORE the response is sent (the
    default "request" scope commits after it: a client that submits and immediately reads back could
    miss its own write)."""
    s = get_db().get_session()
    try:
        yield s
        s.commit()
    except BaseException:
        s.rollback()
        raise
    finally:
        s.close()
