"""Schema migrations (reference: ``src/tests/_internal/server/test_migrations.py``)."""

from sqlalchemy import inspect, text

from dstack_amd.server.db import Database
from dstack_amd.server.migrations import MIGRATIONS, current_version, run_migrations
from dstack_amd.server.models import Base


def test_fresh_database_reaches_latest_version(tmp_path):
    db = Database(f"sqlite:///{tmp_path}/a.db")
    assert run_migrations(db) == len(MIGRATIONS)
    with db.engine.connect() as c:
        tables = set(inspect(c).get_table_names())
        assert set(Base.metadata.tables) <= tables
        assert current_version(c) == len(MIGRATIONS)
    # idempotent: running again applies nothing
    assert run_migrations(db) == len(MIGRATIONS)
    with db.engine.connect() as c:
        assert c.execute(text("SELECT COUNT(*) FROM schema_version")).scalar() == len(MIGRATIONS)


def test_old_database_gets_additive_migrations(tmp_path):
    """A database created by migration 1 without later columns is upgraded in place."""
    db = Database(f"sqlite:///{tmp_path}/b.db")
    with db.engine.begin() as c:
        MIGRATIONS[0](c)
        c.execute(text("ALTER TABLE jobs DROP COLUMN timings"))
        c.execute(text("INSERT INTO schema_version (version, applied_at) VALUES (1, CURRENT_TIMESTAMP)"))
    assert run_migrations(db) == len(MIGRATIONS)
    with db.engine.connect() as c:
        assert "timings" in {col["name"] for col in inspect(c).get_columns("jobs")}
