"""Versioned schema migrations (replaces the reference's 57 alembic revisions,
``S/migrations/versions/*``, 41 of which carry ``op.execute`` data steps).

Model (alembic's, without alembic):

* ``MIGRATIONS[0]`` is the baseline.  A FRESH database (no ``schema_version`` table) is created
  from the ORM metadata in one step and stamped with the latest version -- the later migrations
  describe how OLDER databases reach that schema, they never run on a new one.
* Every later migration is a list of operations (or a plain ``fn(conn)``) applied once, in order,
  inside one transaction with the version bump, to databases at an earlier version.  Each may
  assume exactly the schema its predecessor left.
* Operations (both dialects: SQLite >= 3.35 and Postgres):
  ``add_column``, ``drop_column``, ``rename_column``, ``alter_column_type`` (with a ``using``
  conversion expression), ``rename_table``, ``create_index`` / ``drop_index``, ``backfill``
  (UPDATE ... SET ... WHERE ...), ``rename_enum_value`` (enum-like VARCHAR columns: the server
  stores enums as strings, so a value rename is data, and adding a value needs no DDL -- unlike the
  reference's Postgres ENUM types that need ALTER TYPE) and ``run_python`` (arbitrary data step
  over the connection).
* SQLite has no ALTER COLUMN TYPE: the column is renamed aside, re-added with the new type, filled
  through ``using`` and the old one dropped; indexes on the column are dropped first and re-created
  after.  No table rebuild (a DROP TABLE of a parent would cascade through ON DELETE).

A process-wide lock (plus SQLite's own write lock, or a Postgres advisory lock shared by server
replicas) serialises concurrent server starts.
"""

from __future__ import annotations

import threading
from typing import Callable, Dict, List, Optional, Sequence, Union

from sqlalchemy import inspect, text

from dstack_amd.server.models import Base


class MigrationError(RuntimeError):
    """An operation that cannot be applied safely to this database (nothing of it was applied)."""

_lock = threading.Lock()


def _q(name: str) -> str:
    return '"' + name.replace('"', '""') + '"'


def _columns(conn, table: str) -> List[str]:
    return [c["name"] for c in inspect(conn).get_columns(table)]


def _indexes_on(conn, table: str, column: str) -> List[dict]:
    return [ix for ix in inspect(conn).get_indexes(table) if column in (ix.get("column_names") or [])]


class Op:
    """One schema or data step; ``sql(dialect)`` is what it executes where that is static."""

    def apply(self, conn) -> None:  # pragma: no cover - interface
        raise NotImplementedError

    def __call__(self, conn) -> None:
        self.apply(conn)


class add_column(Op):
    def __init__(self, table: str, column: str, ddl: str):
        self.table, self.column, self.ddl = table, column, ddl

    def apply(self, conn):
        if self.column not in _columns(conn, self.table):
            conn.execute(text(f"ALTER TABLE {_q(self.table)} ADD COLUMN {_q(self.column)} {self.ddl}"))


class drop_column(Op):
    def __init__(self, table: str, column: str):
        self.table, self.column = table, column

    def apply(self, conn):
        if self.column not in _columns(conn, self.table):
            return
        for ix in _indexes_on(conn, self.table, self.column):  # SQLite refuses to drop an indexed column
            conn.execute(text(f"DROP INDEX {_q(ix['name'])}"))
        conn.execute(text(f"ALTER TABLE {_q(self.table)} DROP COLUMN {_q(self.column)}"))


class rename_column(Op):
    def __init__(self, table: str, old: str, new: str):
        self.table, self.old, self.new = table, old, new

    def apply(self, conn):
        conn.execute(text(f"ALTER TABLE {_q(self.table)} RENAME COLUMN {_q(self.old)} TO {_q(self.new)}"))


class rename_table(Op):
    def __init__(self, old: str, new: str):
        self.old, self.new = old, new

    def apply(self, conn):
        conn.execute(text(f"ALTER TABLE {_q(self.old)} RENAME TO {_q(self.new)}"))


class create_index(Op):
    def __init__(self, name: str, table: str, columns: Sequence[str], unique: bool = False):
        self.name, self.table, self.columns, self.unique = name, table, list(columns), unique

    def apply(self, conn):
        cols = ", ".join(_q(c) for c in self.columns)
        conn.execute(text(f"CREATE {'UNIQUE ' if self.unique else ''}INDEX IF NOT EXISTS {_q(self.name)} "
                          f"ON {_q(self.table)} ({cols})"))


class drop_index(Op):
    def __init__(self, name: str):
        self.name = name

    def apply(self, conn):
        conn.execute(text(f"DROP INDEX IF EXISTS {_q(self.name)}"))


class alter_column_type(Op):
    """``using``: SQL template over ``{col}`` (the quoted column) giving the new value, e.g.
    ``CAST(trim({col}) AS INTEGER)``; default a plain CAST to ``new_type``.

    On SQLite (no ALTER COLUMN) the column is renamed aside, re-added and converted: its NOT NULL
    and DEFAULT are carried over and its indexes re-created.  Refused there (a table rebuild through
    ``run_python`` is needed instead): primary-key, foreign-key and inline-UNIQUE columns, and NOT
    NULL columns without a DEFAULT (SQLite cannot add those).  CHECK constraints that name the
    column are not carried over."""

    def __init__(self, table: str, column: str, new_type: str, using: Optional[str] = None):
        self.table, self.column, self.new_type = table, column, new_type
        self.using = using or ("CAST({col} AS %s)" % new_type)

    def apply(self, conn):
        t, c = _q(self.table), _q(self.column)
        if conn.dialect.name == "postgresql":
            conn.execute(text(f"ALTER TABLE {t} ALTER COLUMN {c} TYPE {self.new_type} "
                              f"USING {self.using.format(col=c)}"))
            return
        # SQLite: aside, re-add, convert, drop -- constraints carried, indexes re-created
        info = {r[1]: r for r in conn.execute(text(f"PRAGMA table_info({t})")).fetchall()}
        if self.column not in info:
            raise MigrationError(f"{self.table}.{self.column}: no such column")
        _, _, _, notnull, default, pk = info[self.column]
        fks = [r for r in conn.execute(text(f"PRAGMA foreign_key_list({t})")).fetchall() if r[3] == self.column]
        auto_unique = [ix for ix in conn.execute(text(f"PRAGMA index_list({t})")).fetchall()
                       if ix[1].startswith("sqlite_autoindex_") and
                       [r[2] for r in conn.execute(text(f"PRAGMA index_info({_q(ix[1])})")).fetchall()] == [self.column]]
        if pk or fks or auto_unique:
            what = "primary-key" if pk else "foreign-key" if fks else "UNIQUE"
            raise MigrationError(f"{self.table}.{self.column}: alter_column_type cannot retype a {what} column on "
                                 "SQLite; rebuild the table with run_python")
        if notnull and default is None:
            raise MigrationError(f"{self.table}.{self.column}: NOT NULL without DEFAULT cannot be re-added on "
                                 "SQLite; rebuild the table with run_python")
        decl = self.new_type + (" NOT NULL" if notnull else "") + (f" DEFAULT {default}" if default is not None else "")
        indexes = _indexes_on(conn, self.table, self.column)
        for ix in indexes:
            conn.execute(text(f"DROP INDEX {_q(ix['name'])}"))
        aside = _q(f"_old_{self.column}")
        conn.execute(text(f"ALTER TABLE {t} RENAME COLUMN {c} TO {aside}"))
        conn.execute(text(f"ALTER TABLE {t} ADD COLUMN {c} {decl}"))
        conn.execute(text(f"UPDATE {t} SET {c} = {self.using.format(col=aside)}"))
        conn.execute(text(f"ALTER TABLE {t} DROP COLUMN {aside}"))
        for ix in indexes:
            create_index(ix["name"], self.table, ix["column_names"], bool(ix.get("unique"))).apply(conn)


class backfill(Op):
    """``UPDATE table SET <set_sql> [WHERE <where>]`` with bound ``params``."""

    def __init__(self, table: str, set_sql: str, where: Optional[str] = None, params: Optional[Dict] = None):
        self.table, self.set_sql, self.where, self.params = table, set_sql, where, params or {}

    def apply(self, conn):
        sql = f"UPDATE {_q(self.table)} SET {self.set_sql}" + (f" WHERE {self.where}" if self.where else "")
        conn.execute(text(sql), self.params)


class rename_enum_value(Op):
    def __init__(self, table: str, column: str, old: str, new: str):
        self.table, self.column, self.old, self.new = table, column, old, new

    def apply(self, conn):
        backfill(self.table, f"{_q(self.column)} = :new", f"{_q(self.column)} = :old",
                 {"new": self.new, "old": self.old}).apply(conn)


class run_python(Op):
    def __init__(self, fn: Callable, doc: str = ""):
        self.fn, self.doc = fn, doc

    def apply(self, conn):
        self.fn(conn)


Migration = Union[Callable, Sequence[Op]]


def _m0001_initial(conn):
    Base.metadata.create_all(conn)


def _apply(mig: Migration, conn) -> None:
    if callable(mig):
        mig(conn)
    else:
        for op in mig:
            op.apply(conn)


MIGRATIONS: List[Migration] = [
    _m0001_initial,
    # columns added after the first release (databases created before them)
    [add_column("jobs", "timings", "TEXT")],
    [add_column("job_metrics_points", "gpus_extra", "TEXT")],
    [add_column("instances", "deploy_owner", "VARCHAR(100)")],
    [add_column("instances", "deploy_started_at", "TIMESTAMP")],
    # the gpu_util autoscaler and `dstack stats` read each job's newest samples: (job, time) index
    [create_index("ix_job_metrics_points_job_ts", "job_metrics_points", ["job_id", "timestamp_micro"])],
]


def current_version(conn) -> int:
    if "schema_version" not in inspect(conn).get_table_names():
        return 0
    row = conn.execute(text("SELECT MAX(version) FROM schema_version")).scalar()
    return int(row or 0)


MIGRATIONS_LOCK_NAME = "dstack_migrations"


def run_migrations(db, migrations: Optional[List[Migration]] = None, metadata=None) -> int:
    """Bring the database to the latest version; returns it.  A fresh database gets the current
    schema from ``metadata`` (default: the ORM's) and is stamped with the latest version; an older
    one runs every pending migration.  All of it is ONE transaction: a failing step leaves the
    database at its previous version (on SQLite too -- pysqlite would run DDL outside a transaction,
    so the migration connection issues its own BEGIN IMMEDIATE).  Server replicas sharing a Postgres
    database serialise on a transaction-scoped advisory lock (reference ``S/db.py:75-82``: alembic
    under an advisory lock)."""
    from dstack_amd.server.services.locking import ADVISORY_XACT_LOCK_SQL, advisory_key

    migrations = MIGRATIONS if migrations is None else migrations
    metadata = Base.metadata if metadata is None else metadata
    with _lock:
        with db.engine.connect() as conn:
            sqlite = conn.dialect.name == "sqlite"
            dbapi = conn.connection.driver_connection if sqlite else None
            prev = dbapi.isolation_level if sqlite else None
            try:
                if sqlite:
                    dbapi.isolation_level = None  # we open and close the transaction ourselves
                    conn.exec_driver_sql("BEGIN IMMEDIATE")
                elif conn.dialect.name == "postgresql":
                    conn.execute(text(ADVISORY_XACT_LOCK_SQL), {"k": advisory_key(MIGRATIONS_LOCK_NAME)})
                v = _migrate(conn, migrations, metadata)
                conn.commit()
                return v
            except BaseException:
                conn.rollback()
                raise
            finally:
                if sqlite:
                    dbapi.isolation_level = prev


def _migrate(conn, migrations: List[Migration], metadata) -> int:
    latest = len(migrations)
    v = current_version(conn)
    tables = set(inspect(conn).get_table_names())
    if not tables:  # fresh: the current schema in one step
        metadata.create_all(conn)
        _stamp(conn, latest)
        return latest
    if "schema_version" not in tables:  # created before versioning: the baseline
        metadata.create_all(conn)
        _stamp(conn, 1)
        v = 1
    for i, mig in enumerate(migrations, start=1):
        if i <= v:
            continue
        _apply(mig, conn)
        _stamp(conn, i)
        v = i
    return v


def _stamp(conn, version: int) -> None:
    if "schema_version" not in inspect(conn).get_table_names():
        conn.execute(text("CREATE TABLE schema_version (version INTEGER PRIMARY KEY, applied_at TIMESTAMP)"))
    conn.execute(text("INSERT INTO schema_version (version, applied_at) VALUES (:v, CURRENT_TIMESTAMP)"),
                 {"v": version})
