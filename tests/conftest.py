import os
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# isolate every server/CLI test from the real ~/.dstack before any dstack_amd module reads settings
_TMP_HOME = tempfile.mkdtemp(prefix="dstack-amd-tests-")
os.environ.setdefault("DSTACK_DIR", os.path.join(_TMP_HOME, "dstack"))
os.environ["DSTACK_SERVER_NO_CLIENT_CONFIG"] = "1"
# cloud backends plan from the offline catalog unless a test opts into live listings
# (tests/test_catalog.py); the catalog cache never touches the real ~/.dstack
os.environ["DSTACK_CATALOG_OFFLINE_ONLY"] = "1"
os.environ["DSTACK_CATALOG_CACHE_DIR"] = os.path.join(_TMP_HOME, "catalog")

ADMIN_TOKEN = "test-admin-token"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    return torch.device("cuda", 0)


@pytest.fixture
def db():
    """Fresh in-memory database with migrations applied and the default admin/project created."""
    from dstack_amd.server import db as db_mod
    from dstack_amd.server.app import init_server_state

    prev = db_mod._db
    d = db_mod.Database("sqlite://")
    db_mod.override_db(d)
    init_server_state(ADMIN_TOKEN)
    yield d
    d.engine.dispose()
    db_mod.override_db(prev)


@pytest.fixture
def session(db):
    from dstack_amd.server.db import session_scope

    with session_scope() as s:
        yield s


@pytest.fixture
def client(db):
    """FastAPI TestClient without background reconcilers (tests drive them explicitly)."""
    from fastapi.testclient import TestClient

    from dstack_amd.server.app import create_app

    app = create_app(start_background=False)
    with TestClient(app) as c:
        c.headers.update({"Authorization": f"Bearer {ADMIN_TOKEN}"})
        yield c
