"""FastAPI dependencies (reference: ``S/deps.py``)."""

from __future__ import annotations

from typing import Iterator

from sqlalchemy.orm import Session

from dstack_amd.server.db import get_db


def get_session() -> Iterator[Session]:
    s = get_db().get_session()
    try:
        yield s
        s.commit()
    except BaseException:
        s.rollback()
        raise
    finally:
        s.close()
