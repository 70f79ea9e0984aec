"""Postgres multi-replica paths (reference: ``S/services/locking.py``, ``contributing/LOCKING.md``).
No Postgres server or driver exists in this image, so the statements are checked by compiling them
with SQLAlchemy's postgresql dialect, and the dialect switch is exercised with a stand-in session."""

from unittest import mock

from sqlalchemy.dialects import postgresql

from dstack_amd.server.models import JobModel
from dstack_amd.server.services import locking


def _pg_session(result=1):
    s = mock.Mock()
    s.get_bind.return_value.dialect.name = "postgresql"
    s.execute.return_value.scalar_one_or_none.return_value = result
    return s


def test_claim_row_statement_is_skip_locked():
    sql = str(locking.claim_row_stmt(JobModel, "x").compile(dialect=postgresql.dialect()))
    assert "FOR UPDATE SKIP LOCKED" in sql and "jobs.id" in sql


def test_claim_row_postgres_and_sqlite():
    assert locking.claim_row(_pg_session(result=1), JobModel, "a") is True
    assert locking.claim_row(_pg_session(result=None), JobModel, "a") is False  # held by another replica
    sq = mock.Mock()
    sq.get_bind.return_value.dialect.name = "sqlite"
    assert locking.claim_row(sq, JobModel, "a") is True
    sq.execute.assert_not_called()


def test_db_advisory_lock_uses_stable_key():
    s = _pg_session()
    with locking.db_advisory_lock(s, "run_names_p1"):
        pass
    stmt, params = s.execute.call_args[0]
    assert "pg_advisory_xact_lock" in str(stmt)
    assert params["k"] == locking.advisory_key("run_names_p1")
    assert locking.advisory_key("a") != locking.advisory_key("b")
    assert -(2**63) <= locking.advisory_key("a") < 2**63


def test_claim_and_process_skips_rows_locked_elsewhere(db):
    from dstack_amd.server.background import common

    seen = []
    with mock.patch.object(common, "claim_row", side_effect=lambda s, m, i: i != "b"):
        common.claim_and_process("jobs", lambda s: ["a", "b", "c"], lambda s, i: seen.append(i), batch=5)
    assert seen == ["a", "c"]


def test_postgres_engine_options():
    from dstack_amd.server import db as dbmod

    with mock.patch.object(dbmod, "create_engine") as ce, mock.patch.object(dbmod.event, "listen"):
        dbmod.Database("postgresql+psycopg://u:p@h/d")
    kwargs = ce.call_args.kwargs
    assert kwargs["pool_pre_ping"] and kwargs["pool_size"] > 0 and "connect_args" not in kwargs
