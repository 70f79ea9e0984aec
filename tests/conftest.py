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
# placeholder cloud credentials are not sent to the clouds (tests/test_backends_api.py opts in)
os.environ["DSTACK_SKIP_BACKEND_VALIDATION"] = "1"

# No test touches the network (the reference runs pytest-socket with --allow-hosts=127.0.0.1):
# connections and name lookups are limited to loopback and unix sockets in the test process.
import socket as _socket  # noqa: E402

_LOCAL = {"127.0.0.1", "::1", "localhost", "0.0.0.0", "::", "", None}
_orig_connect, _orig_connect_ex = _socket.socket.connect, _socket.socket.connect_ex
_orig_getaddrinfo = _socket.getaddrinfo


def _check_addr(sock, addr):
    if sock.family in (_socket.AF_INET, _socket.AF_INET6) and isinstance(addr, tuple) and addr[0] not in _LOCAL:
        raise ConnectionRefusedError(f"network access disabled in tests: {addr[0]}")


def _guarded_connect(self, addr):
    _check_addr(self, addr)
    return _orig_connect(self, addr)


def _guarded_connect_ex(self, addr):
    _check_addr(self, addr)
    return _orig_connect_ex(self, addr)


def _guarded_getaddrinfo(host, *a, **kw):
    h = host.decode() if isinstance(host, bytes) else host
    if h not in _LOCAL and not (isinstance(h, str) and h.startswith("127.")):
        raise _socket.gaierror(_socket.EAI_NONAME, f"name resolution disabled in tests: {h}")
    return _orig_getaddrinfo(host, *a, **kw)


if os.environ.get("DSTACK_TESTS_ALLOW_NETWORK") != "1":
    _socket.socket.connect = _guarded_connect
    _socket.socket.connect_ex = _guarded_connect_ex
    _socket.getaddrinfo = _guarded_getaddrinfo

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
