"""Server settings under the reference's environment-variable names (reference:
``src/dstack/_internal/server/settings.py``): each switch changes the behaviour it names."""

import pytest

from dstack_amd.server import settings


def _service(name="svc", **kw):
    conf = {"type": "service", "commands": ["python3 -m http.server 8000"], "port": 8000}
    conf.update(kw)
    return {"run_spec": {"run_name": name, "repo_id": "virt", "repo_data": {"repo_type": "virtual"},
                         "configuration": conf, "ssh_key_pub": ""}}


def test_default_creds_disabled(client, monkeypatch):
    body = {"type": "aws", "regions": ["us-east-1"], "creds": {"type": "default"}}
    monkeypatch.setattr(settings, "DEFAULT_CREDS_DISABLED", True)
    r = client.post("/api/project/main/backends/create", json=body)
    assert r.status_code == 400 and "Default credentials are forbidden" in r.text
    monkeypatch.setattr(settings, "DEFAULT_CREDS_DISABLED", False)
    assert client.post("/api/project/main/backends/create", json=body).status_code == 200


def test_forbid_services_without_gateway(client, monkeypatch):
    client.post("/api/project/main/repos/init", json={"repo_id": "virt", "repo_info": {"repo_type": "virtual"}})
    monkeypatch.setattr(settings, "FORBID_SERVICES_WITHOUT_GATEWAY", True)
    r = client.post("/api/project/main/runs/submit", json=_service())
    assert r.status_code == 400 and "forbids services without a gateway" in r.text
    assert client.post("/api/project/main/runs/get", json={"run_name": "svc"}).status_code == 400
    monkeypatch.setattr(settings, "FORBID_SERVICES_WITHOUT_GATEWAY", False)
    r = client.post("/api/project/main/runs/submit", json=_service())
    assert r.status_code == 200, r.text
    assert r.json()["service"]["url"] == "/proxy/services/main/svc/"


def test_user_project_default_quota(client, monkeypatch):
    monkeypatch.setattr(settings, "USER_PROJECT_DEFAULT_QUOTA", 1)
    u = client.post("/api/users/create", json={"username": "quota-user"}).json()
    h = {"Authorization": f"Bearer {u['creds']['token']}"}
    assert client.post("/api/projects/create", json={"project_name": "q1"}, headers=h).status_code == 200
    r = client.post("/api/projects/create", json={"project_name": "q2"}, headers=h)
    assert r.status_code == 400 and "quota" in r.text


def test_force_bridge_network(monkeypatch):
    from dstack_amd.core.models.backends import BackendType
    from dstack_amd.core.models.instances import (
        InstanceAvailability,
        InstanceOfferWithAvailability,
        InstanceType,
        Resources,
    )
    from dstack_amd.core.models.runs import NetworkMode
    from dstack_amd.server.background.tasks.process_submitted_jobs import _runtime_data

    offer = InstanceOfferWithAvailability(
        backend=BackendType.LOCAL, region="local", price=0.0, availability=InstanceAvailability.AVAILABLE,
        instance=InstanceType(name="local", resources=Resources(cpus=8, memory_mib=65536, gpus=[], spot=False)))
    assert _runtime_data(offer, None, None).network_mode == NetworkMode.HOST
    monkeypatch.setattr(settings, "FORCE_BRIDGE_NETWORK", True)
    assert _runtime_data(offer, None, None).network_mode == NetworkMode.BRIDGE


@pytest.mark.parametrize("mode", ["fresh", "other-server", "other-server-yes", "no"])
def test_default_project_written_to_cli_config(tmp_path, monkeypatch, mode):
    """``dstack server`` makes its project the CLI default when the CLI has none; another server's
    default project is kept unless DSTACK_UPDATE_DEFAULT_PROJECT; DSTACK_DO_NOT_UPDATE_DEFAULT_PROJECT
    never writes (reference ``core/services/configs/__init__.py:update_default_project``)."""
    from dstack_amd.core.services.configs import ConfigManager
    from dstack_amd.server.app import _write_client_config

    monkeypatch.setenv("DSTACK_DIR", str(tmp_path))
    monkeypatch.delenv("DSTACK_SERVER_NO_CLIENT_CONFIG", raising=False)
    monkeypatch.setattr("sys.stdin.isatty", lambda: False, raising=False)
    if mode != "fresh":
        cm = ConfigManager()
        cm.configure_project("main", "http://other:3000", "tok0", default=True)
        cm.save()
    monkeypatch.setattr(settings, "UPDATE_DEFAULT_PROJECT", mode == "other-server-yes")
    monkeypatch.setattr(settings, "DO_NOT_UPDATE_DEFAULT_PROJECT", mode == "no")
    _write_client_config("http://127.0.0.1:3000", "tok1")
    p = ConfigManager().get_project_config()
    if mode in ("fresh", "other-server-yes"):
        assert (p.url, p.token) == ("http://127.0.0.1:3000", "tok1")
    else:
        assert (p.url, p.token) == ("http://other:3000", "tok0")


def test_server_config_disabled(tmp_path, monkeypatch):
    from dstack_amd.server import db as db_mod
    from dstack_amd.server.app import init_server_state
    from dstack_amd.server.services import permissions

    cfg = tmp_path / "config.yml"
    cfg.write_text("default_permissions:\n  allow_non_admins_create_projects: false\n")
    monkeypatch.setattr(settings, "SERVER_CONFIG_FILE_PATH", cfg)
    prev = db_mod._db
    try:
        for disabled, expect in ((True, True), (False, False)):
            monkeypatch.setattr(settings, "SERVER_CONFIG_DISABLED", disabled)
            db_mod.override_db(db_mod.Database("sqlite://"))
            init_server_state("tok")
            assert permissions.get_default_permissions().allow_non_admins_create_projects is expect
    finally:
        permissions.set_default_permissions(None)
        db_mod.override_db(prev)
