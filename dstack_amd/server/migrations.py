"""Versioned schema migrations (replaces the reference's 57 alembic revisions,
``S/migrations/versions/*``).

Migration 1 creates the full current schema from the ORM metadata.  Later migrations are plain
functions ``(connection) -> None`` appended to ``MIGRATIONS``; each runs once, in order, inside a
transaction, and the applied version is recorded in ``schema_version``.  A process-wide lock
(plus SQLite's own write lock) serialises concurrent server starts.
"""

from __future__ import annotations

import threading
from typing import Callable, List

from sqlalchemy import inspect, text

from dstack_amd.server.models import Base

_lock = threading.Lock()


def _m0001_initial(conn):
    Base.metadata.create_all(conn)


def _add_column(table: str, column: str, ddl: str):
    def mig(conn):
        cols = {c["name"] for c in inspect(conn).get_columns(table)}
        if column not in cols:
            conn.execute(text(f"ALTER TABLE {table} ADD COLUMN {column} {ddl}"))

    return mig


MIGRATIONS: List[Callable] = [
    _m0001_initial,
    # example of an additive migration kept for databases created before the column existed
    _add_column("jobs", "timings", "TEXT"),
    _add_column("job_metrics_points", "gpus_extra", "TEXT"),
    _add_column("instances", "deploy_owner", "VARCHAR(100)"),
    _add_column("instances", "deploy_started_at", "TIMESTAMP"),
]


def current_version(conn) -> int:
    if "schema_version" not in inspect(conn).get_table_names():
        return 0
    row = conn.execute(text("SELECT MAX(version) FROM schema_version")).scalar()
    return int(row or 0)


MIGRATIONS_LOCK_NAME = "dstack_migrations"


def run_migrations(db) -> int:
    """Apply pending migrations.  Server replicas sharing a Postgres database serialise on a
    transaction-scoped advisory lock (reference ``S/db.py:75-82``: alembic under an advisory lock)."""
    from dstack_amd.server.services.locking import ADVISORY_XACT_LOCK_SQL, advisory_key

    with _lock:
        with db.engine.begin() as conn:
            if conn.dialect.name == "postgresql":
                conn.execute(text(ADVISORY_XACT_LOCK_SQL), {"k": advisory_key(MIGRATIONS_LOCK_NAME)})
            v = current_version(conn)
            for i, mig in enumerate(MIGRATIONS, start=1):
                if i <= v:
                    continue
                mig(conn)
                conn.execute(text("INSERT INTO schema_version (version, applied_at) VALUES (:v, CURRENT_TIMESTAMP)"),
                             {"v": i})
                v = i
            return v
