"""Database layer: SQLAlchemy 2.0 ORM over SQLite (WAL) or Postgres — reference: ``S/db.py:16-106``.

The MI355X build runs the control plane synchronously: request handlers and reconciler tasks run
in worker threads, each with its own short ``Session``.  SQLite is opened in WAL mode with a 30 s
busy timeout and foreign keys on; schema evolution uses the versioned migrations in
``server/migrations.py`` (no alembic in this image).  With ``DSTACK_DATABASE_URL=postgresql://...``
several server replicas share the database: reconcilers claim rows with ``FOR UPDATE SKIP LOCKED``
and named operations/migrations take ``pg_advisory_xact_lock`` (``services/locking.py``).  The
Postgres driver (psycopg) is not part of this image, so that path is covered by SQL-compilation
tests only.
"""

from __future__ import annotations

import contextlib
import threading
from typing import Iterator, Optional

from sqlalchemy import create_engine, event
from sqlalchemy.engine import Engine
from sqlalchemy.orm import Session, sessionmaker
from sqlalchemy.pool import StaticPool

from dstack_amd.server import settings


class Database:
    def __init__(self, url: str, echo: bool = False):
        self.url = url
        kwargs: dict = {"echo": echo, "future": True}
        if url.startswith("sqlite"):
            kwargs["connect_args"] = {"check_same_thread": False, "timeout": 30}
            if url in ("sqlite://", "sqlite:///:memory:"):
                kwargs["poolclass"] = StaticPool
        else:  # postgresql(+psycopg)://: several server replicas may share the database
            kwargs["pool_size"] = settings.DB_POOL_SIZE
            kwargs["max_overflow"] = settings.DB_MAX_OVERFLOW
            kwargs["pool_pre_ping"] = True
        self.engine: Engine = create_engine(url, **kwargs)
        if url.startswith("sqlite"):
            event.listen(self.engine, "connect", _sqlite_pragmas)
        self.session_maker = sessionmaker(bind=self.engine, expire_on_commit=False, future=True)
        # serialises writers on SQLite (a single writer at a time is what SQLite allows anyway);
        # avoids "database is locked" storms under many reconciler threads
        self.write_lock = threading.RLock() if url.startswith("sqlite") else None

    @property
    def dialect_name(self) -> str:
        return self.engine.dialect.name

    def get_session(self) -> Session:
        return self.session_maker()


def _sqlite_pragmas(dbapi_conn, _):
    cur = dbapi_conn.cursor()
    cur.execute("PRAGMA journal_mode=WAL;")
    cur.execute("PRAGMA foreign_keys=ON;")
    cur.execute("PRAGMA synchronous=NORMAL;")
    cur.execute("PRAGMA busy_timeout=30000;")
    cur.close()


_db: Optional[Database] = None


def get_db() -> Database:
    global _db
    if _db is None:
        if settings.DATABASE_URL.startswith("sqlite:///"):
            from pathlib import Path

            Path(settings.DATABASE_URL[len("sqlite:///"):]).parent.mkdir(parents=True, exist_ok=True)
        _db = Database(settings.DATABASE_URL, echo=settings.SQL_ECHO_ENABLED)
    return _db


def override_db(db: Database):
    global _db
    _db = db


@contextlib.contextmanager
def session_scope(db: Optional[Database] = None) -> Iterator[Session]:
    db = db or get_db()
    s = db.get_session()
    try:
        yield s
        s.commit()
    except BaseException:
        s.rollback()
        raise
    finally:
        s.close()


def migrate(db: Optional[Database] = None):
    from dstack_amd.server.migrations import run_migrations

    run_migrations(db or get_db())
