"""Schema migrations (reference: ``src/tests/_internal/server/test_migrations.py``; the reference's
57 alembic revisions, 41 with ``op.execute`` data steps, ``S/migrations/versions/*``).

* a fresh database gets the current schema in one step, stamped with the latest version;
* a database written at version 1 -- with rows -- is upgraded through renames, a type change with a
  conversion, a backfill, an enum-value rename and a drop of an indexed column, and its data is
  checked afterwards (SQLite here; the Postgres statements are checked by capturing them, there is
  no Postgres server in this image);
* the real chain (``MIGRATIONS``) upgrades a database written before its later steps."""

import sqlite3

import pytest
from sqlalchemy import Column, Integer, MetaData, String, Table, inspect, text

from dstack_amd.server import migrations as m
from dstack_amd.server.db import Database
from dstack_amd.server.migrations import MIGRATIONS, current_version, run_migrations
from dstack_amd.server.models import Base

pytestmark = pytest.mark.skipif(sqlite3.sqlite_version_info < (3, 35), reason="DROP COLUMN needs SQLite 3.35")


def test_fresh_database_reaches_latest_version_in_one_step(tmp_path):
    db = Database(f"sqlite:///{tmp_path}/a.db")
    assert run_migrations(db) == len(MIGRATIONS)
    with db.engine.connect() as c:
        assert set(Base.metadata.tables) <= set(inspect(c).get_table_names())
        assert current_version(c) == len(MIGRATIONS)
        assert c.execute(text("SELECT COUNT(*) FROM schema_version")).scalar() == 1  # stamped, not replayed
        ix = {i["name"] for i in inspect(c).get_indexes("job_metrics_points")}
        assert "ix_job_metrics_points_job_ts" in ix
    assert run_migrations(db) == len(MIGRATIONS)  # idempotent


# ---- a synthetic schema history --------------------------------------------------------------------
V1_DDL = [
    "CREATE TABLE widgets (id INTEGER PRIMARY KEY, name VARCHAR(50), size_txt TEXT, color VARCHAR(10), "
    "status VARCHAR(20))",
    "CREATE INDEX ix_widgets_color ON widgets (color)",
    "CREATE INDEX ix_widgets_size ON widgets (size_txt)",
    "CREATE TABLE schema_version (version INTEGER PRIMARY KEY, applied_at TIMESTAMP)",
]


def _v1(conn):
    for ddl in V1_DDL:
        conn.execute(text(ddl))


CHAIN = [
    _v1,
    [m.rename_column("widgets", "name", "title")],
    [m.alter_column_type("widgets", "size_txt", "INTEGER", using="CAST(trim({col}) AS INTEGER)"),
     m.rename_column("widgets", "size_txt", "size")],
    [m.add_column("widgets", "area", "INTEGER"), m.backfill("widgets", "area = size * size", "area IS NULL")],
    [m.rename_enum_value("widgets", "status", "Pending", "pending"),
     m.rename_enum_value("widgets", "status", "Done", "done")],
    [m.drop_column("widgets", "color")],
    [m.rename_table("widgets", "gadgets")],
]


def _final_metadata():
    md = MetaData()
    Table("gadgets", md, Column("id", Integer, primary_key=True), Column("title", String(50)),
          Column("size", Integer), Column("status", String(20)), Column("area", Integer))
    Table("schema_version", md, Column("version", Integer, primary_key=True), Column("applied_at", String))
    return md


def test_v1_database_with_rows_is_upgraded_through_every_kind_of_step(tmp_path):
    db = Database(f"sqlite:///{tmp_path}/w.db")
    with db.engine.begin() as c:
        _v1(c)
        c.execute(text("INSERT INTO schema_version VALUES (1, CURRENT_TIMESTAMP)"))
        c.execute(text("INSERT INTO widgets VALUES (1, 'a', ' 12', 'RED', 'Pending'), (2, 'b', '7', 'BLUE', 'Done'),"
                       " (3, 'c', '3', NULL, 'Failed')"))
    assert run_migrations(db, CHAIN, _final_metadata()) == len(CHAIN)
    with db.engine.connect() as c:
        insp = inspect(c)
        assert "widgets" not in insp.get_table_names()
        cols = {col["name"]: str(col["type"]) for col in insp.get_columns("gadgets")}
        assert set(cols) == {"id", "title", "size", "status", "area"} and cols["size"] == "INTEGER"
        assert {i["name"]: i["column_names"] for i in insp.get_indexes("gadgets")} == {"ix_widgets_size": ["size"]}
        rows = c.execute(text("SELECT id, title, size, typeof(size), area, status FROM gadgets ORDER BY id")).all()
        assert rows == [(1, "a", 12, "integer", 144, "pending"), (2, "b", 7, "integer", 49, "done"),
                        (3, "c", 3, "integer", 9, "Failed")]
        assert [r[0] for r in c.execute(text("SELECT version FROM schema_version ORDER BY version"))] == \
            list(range(1, len(CHAIN) + 1))
    # a fresh database of the same history is the final schema directly
    fresh = Database(f"sqlite:///{tmp_path}/f.db")
    assert run_migrations(fresh, CHAIN, _final_metadata()) == len(CHAIN)
    with fresh.engine.connect() as c:
        assert set(inspect(c).get_table_names()) == {"gadgets", "schema_version"}


def test_a_failing_step_rolls_the_whole_migration_back(tmp_path):
    db = Database(f"sqlite:///{tmp_path}/r.db")
    with db.engine.begin() as c:
        _v1(c)
        c.execute(text("INSERT INTO schema_version VALUES (1, CURRENT_TIMESTAMP)"))
    bad = [CHAIN[0], [m.rename_column("widgets", "name", "title"), m.rename_column("widgets", "nope", "x")]]
    with pytest.raises(Exception):
        run_migrations(db, bad, _final_metadata())
    with db.engine.connect() as c:
        assert current_version(c) == 1
        assert "name" in {col["name"] for col in inspect(c).get_columns("widgets")}


class _PgConn:
    """Stand-in Postgres connection: records the statements the operations emit."""

    class dialect:
        name = "postgresql"

    def __init__(self):
        self.sql = []

    def execute(self, stmt, params=None):
        self.sql.append((str(stmt), params))


def test_postgres_statements():
    c = _PgConn()
    m.alter_column_type("widgets", "size_txt", "INTEGER", using="CAST(trim({col}) AS INTEGER)").apply(c)
    m.rename_column("widgets", "name", "title").apply(c)
    m.rename_enum_value("runs", "status", "Pending", "pending").apply(c)
    m.rename_table("widgets", "gadgets").apply(c)
    m.create_index("ix_a", "gadgets", ["status", "id"], unique=True).apply(c)
    got = [s for s, _ in c.sql]
    assert got[0] == 'ALTER TABLE "widgets" ALTER COLUMN "size_txt" TYPE INTEGER USING CAST(trim("size_txt") AS INTEGER)'
    assert got[1] == 'ALTER TABLE "widgets" RENAME COLUMN "name" TO "title"'
    assert got[2] == 'UPDATE "runs" SET "status" = :new WHERE "status" = :old'
    assert c.sql[2][1] == {"new": "pending", "old": "Pending"}
    assert got[3] == 'ALTER TABLE "widgets" RENAME TO "gadgets"'
    assert got[4] == 'CREATE UNIQUE INDEX IF NOT EXISTS "ix_a" ON "gadgets" ("status", "id")'


def test_real_chain_upgrades_a_database_written_before_its_later_steps(tmp_path):
    """Version 1 of the real schema: the ORM schema without the columns and index migrations 2-6
    added, holding a job with metrics; after the upgrade the rows are intact and the new columns
    and index exist."""
    db = Database(f"sqlite:///{tmp_path}/b.db")
    with db.engine.begin() as c:
        c.exec_driver_sql("PRAGMA foreign_keys=OFF")  # a metrics row without its job/run/project chain
        Base.metadata.create_all(c)
        c.execute(text("DROP INDEX ix_job_metrics_points_job_ts"))
        for table, col in [("jobs", "timings"), ("job_metrics_points", "gpus_extra"), ("instances", "deploy_owner"),
                           ("instances", "deploy_started_at")]:
            c.execute(text(f"ALTER TABLE {table} DROP COLUMN {col}"))
        c.execute(text("INSERT INTO schema_version (version, applied_at) VALUES (1, CURRENT_TIMESTAMP)"))
        c.execute(text("INSERT INTO job_metrics_points (id, job_id, timestamp_micro, cpu_usage_micro, "
                       "memory_usage_bytes, memory_working_set_bytes, gpus_memory_usage_bytes, gpus_util_percent) "
                       "VALUES ('m1', 'j1', 5, 1, 2, 3, '[0]', '[97.0]')"))
    assert run_migrations(db) == len(MIGRATIONS)
    with db.engine.connect() as c:
        insp = inspect(c)
        assert "timings" in {col["name"] for col in insp.get_columns("jobs")}
        assert {"deploy_owner", "deploy_started_at"} <= {col["name"] for col in insp.get_columns("instances")}
        assert "ix_job_metrics_points_job_ts" in {i["name"] for i in insp.get_indexes("job_metrics_points")}
        row = c.execute(text("SELECT job_id, gpus_util_percent, gpus_extra FROM job_metrics_points")).one()
        assert tuple(row) == ("j1", "[97.0]", None)


def test_sqlite_retype_keeps_not_null_and_default_and_refuses_key_columns(tmp_path):
    """SQLite's rename-aside retype carries NOT NULL and DEFAULT over (a row inserted afterwards
    without the column still gets the default, a NULL is still refused) and refuses primary-key,
    foreign-key, inline-UNIQUE and NOT-NULL-without-default columns instead of silently dropping
    their constraints."""
    db = Database(f"sqlite:///{tmp_path}/c.db")
    with db.engine.begin() as c:
        c.execute(text("CREATE TABLE parents (id INTEGER PRIMARY KEY)"))
        c.execute(text("CREATE TABLE kids (id INTEGER PRIMARY KEY, n TEXT NOT NULL DEFAULT '7', "
                       "p INTEGER REFERENCES parents(id), code TEXT UNIQUE, req TEXT NOT NULL)"))
        c.execute(text("INSERT INTO parents (id) VALUES (1)"))
        c.execute(text("INSERT INTO kids (id, n, p, code, req) VALUES (1, ' 42 ', 1, 'a', 'x')"))
        m.alter_column_type("kids", "n", "INTEGER", using="CAST(trim({col}) AS INTEGER)").apply(c)
        cols = {r[1]: r for r in c.execute(text("PRAGMA table_info(kids)")).fetchall()}
        assert cols["n"][2] == "INTEGER" and cols["n"][3] == 1 and cols["n"][4] == "'7'"
        assert c.execute(text("SELECT n FROM kids WHERE id = 1")).scalar() == 42
        c.execute(text("INSERT INTO kids (id, req) VALUES (2, 'y')"))
        assert c.execute(text("SELECT n FROM kids WHERE id = 2")).scalar() == 7
        for col, what in (("id", "primary-key"), ("p", "foreign-key"), ("code", "UNIQUE"),
                          ("req", "NOT NULL without DEFAULT")):
            with pytest.raises(m.MigrationError, match=what):
                m.alter_column_type("kids", col, "INTEGER").apply(c)
    with db.engine.begin() as c, pytest.raises(Exception):
        c.execute(text("INSERT INTO kids (id, n, req) VALUES (3, NULL, 'z')"))  # NOT NULL kept
