"""Backend configuration API (reference: ``src/tests/_internal/server/routers/test_backends.py``):
every cloud's YAML contract is validated (type-discriminated configs, ``creds.type`` unions),
secrets are stored apart from the settings and never returned, updates keep omitted credentials,
YAML endpoints, config values from the catalog, project-admin only."""

import json

import pytest
import yaml

from dstack_amd.server.db import session_scope
from dstack_amd.server.models import BackendModel

VALID = {
    "aws": {"type": "aws", "regions": ["us-east-1"], "creds": {"type": "access_key", "access_key": "AKIA",
                                                              "secret_key": "s3"}},
    "azure": {"type": "azure", "tenant_id": "t", "subscription_id": "sub", "locations": ["eastus"],
              "creds": {"type": "client", "client_id": "c", "client_secret": "cs"}},
    "gcp": {"type": "gcp", "project_id": "p", "creds": {"type": "service_account", "filename": "k.json",
                                                        "data": json.dumps({"project_id": "p"})}},
    "oci": {"type": "oci", "regions": ["us-chicago-1"], "creds": {"type": "client", "user": "u", "tenancy": "t",
                                                                   "key_content": "k", "fingerprint": "f",
                                                                   "region": "us-chicago-1"}},
    "lambda": {"type": "lambda", "creds": {"type": "api_key", "api_key": "k"}},
    "vultr": {"type": "vultr", "regions": ["ewr"], "creds": {"type": "api_key", "api_key": "k"}},
    "tensordock": {"type": "tensordock", "creds": {"type": "api_key", "api_key": "k", "api_token": "t"}},
    "cudo": {"type": "cudo", "project_id": "p", "creds": {"type": "api_key", "api_key": "k"}},
    "datacrunch": {"type": "datacrunch", "creds": {"type": "api_key", "client_id": "c", "client_secret": "s"}},
    "nebius": {"type": "nebius", "folder_id": "f", "creds": {"type": "iam_token", "iam_token": "tok"}},
    "runpod": {"type": "runpod", "creds": {"type": "api_key", "api_key": "k"}},
    "vastai": {"type": "vastai", "creds": {"type": "api_key", "api_key": "k"}},
    "kubernetes": {"type": "kubernetes", "networking": {"ssh_host": "1.2.3.4", "ssh_port": 32000},
                   "kubeconfig": {"filename": "kc", "data": "apiVersion: v1\n"}},
}
SECRET_VALUES = {"s3", "cs", "k", "t", "tok", "s", "apiVersion: v1\n"}


@pytest.mark.parametrize("btype", sorted(VALID))
def test_create_each_backend_secrets_kept_apart(client, btype, monkeypatch):
    # placeholder credentials: storage / secret separation is under test, not the cloud's verdict
    # (conftest sets DSTACK_SKIP_BACKEND_VALIDATION for every test)
    r = client.post("/api/project/main/backends/create", json=VALID[btype])
    assert r.status_code == 200, r.text
    info = client.post(f"/api/project/main/backends/{btype}/config_info").json()
    assert info["type"] == btype
    assert "creds" not in info and "kubeconfig" not in info
    flat = json.dumps(info)
    assert not any(f'"{v}"' in flat for v in SECRET_VALUES if len(v) > 1)
    with session_scope() as s:
        row = s.query(BackendModel).filter_by(type=btype).one()
        secrets = json.loads(row.auth)
        assert secrets, "credentials stored in the (encrypted) auth column"
    # the YAML view is the same secret-free config
    y = client.post(f"/api/project/main/backends/{btype}/get_yaml").json()
    assert yaml.safe_load(y["config_yaml"])["type"] == btype


@pytest.mark.parametrize("bad,msg", [
    ({"type": "aws", "creds": {"type": "access_key", "access_key": "A"}}, "secret_key"),
    ({"type": "azure", "subscription_id": "s"}, "tenant_id"),
    ({"type": "gcp", "creds": {"type": "default"}}, "project_id"),
    ({"type": "vultr", "creds": {"type": "password", "api_key": "k"}}, "creds"),
    ({"type": "lambda"}, "creds"),
    ({"type": "runpod", "creds": {"type": "api_key", "api_key": "k"}, "unknown": 1}, "unknown"),
    ({"type": "nosuchcloud"}, "Unknown backend type"),
    ({"type": "local"}, "needs no configuration"),
])
def test_invalid_backend_configs_rejected(client, bad, msg):
    r = client.post("/api/project/main/backends/create", json=bad)
    assert r.status_code == 400, r.text
    assert msg in r.text


def test_duplicate_backend_and_delete(client):
    assert client.post("/api/project/main/backends/create", json=VALID["vultr"]).status_code == 200
    assert client.post("/api/project/main/backends/create", json=VALID["vultr"]).status_code == 400
    client.post("/api/project/main/backends/delete", json={"backends_names": ["vultr"]})
    assert client.post("/api/project/main/backends/vultr/config_info").status_code == 400


def test_update_keeps_omitted_creds(client):
    client.post("/api/project/main/backends/create", json=VALID["aws"])
    r = client.post("/api/project/main/backends/update", json={"type": "aws", "regions": ["us-west-2"]})
    assert r.status_code == 200, r.text
    assert client.post("/api/project/main/backends/aws/config_info").json()["regions"] == ["us-west-2"]
    with session_scope() as s:
        secrets = json.loads(s.query(BackendModel).filter_by(type="aws").one().auth)
        assert secrets["access_key"] == "AKIA" and secrets["secret_key"] == "s3"
    assert client.post("/api/project/main/backends/update", json=VALID["lambda"]).status_code == 400  # not created


def test_yaml_endpoints(client):
    body = {"config_yaml": yaml.safe_dump(VALID["runpod"])}
    assert client.post("/api/project/main/backends/create_yaml", json=body).status_code == 200
    body = {"config_yaml": yaml.safe_dump({"type": "runpod", "regions": ["EU-RO-1"]})}
    assert client.post("/api/project/main/backends/update_yaml", json=body).status_code == 200
    info = client.post("/api/project/main/backends/runpod/config_info").json()
    assert info["regions"] == ["EU-RO-1"]
    bad = {"config_yaml": "- not\n- a mapping\n"}
    assert client.post("/api/project/main/backends/create_yaml", json=bad).status_code == 400


def test_config_values_from_catalog(client):
    r = client.post("/api/backends/config_values", json={"type": "vultr"}).json()
    values = [v["value"] for v in r["regions"]["values"]]
    assert {"ewr", "atl"} <= set(values) and r["regions"]["selected"] == sorted(values)
    r = client.post("/api/backends/config_values", json={"type": "vultr", "regions": ["atl"]}).json()
    assert r["regions"]["selected"] == ["atl"]


def test_backends_are_project_admin_only(client):
    u = client.post("/api/users/create", json={"username": "mallory"}).json()
    h = {"Authorization": f"Bearer {u['creds']['token']}"}
    client.post("/api/projects/main/set_members", json={"members": [
        {"username": "admin", "project_role": "admin"}, {"username": "mallory", "project_role": "user"}]})
    assert client.post("/api/project/main/backends/create", json=VALID["vultr"], headers=h).status_code == 403


def test_configured_backend_offers_in_plan(client):
    """A configured cloud's catalog offers show up in a run plan (MI355X on Vultr bare metal)."""
    client.post("/api/project/main/backends/create", json=VALID["vultr"])
    client.post("/api/project/main/repos/init", json={"repo_id": "virt", "repo_info": {"repo_type": "virtual"}})
    spec = {"run_spec": {"run_name": "plan-mi355x", "repo_id": "virt", "repo_data": {"repo_type": "virtual"},
                         "configuration": {"type": "task", "commands": ["x"], "resources": {"gpu": "MI355X:8"}},
                         "ssh_key_pub": ""}}
    plan = client.post("/api/project/main/runs/get_plan", json=spec).json()
    offers = plan["job_plans"][0]["offers"]
    assert any(o["backend"] == "vultr" and o["instance"]["resources"]["gpus"][0]["name"] == "MI355X" for o in offers)


def test_backend_credentials_validated_on_create(client, monkeypatch):
    """The cloud's verdict on the credentials decides (reference configurators): rejected -> 400
    ``invalid_credentials``; unreachable API (air-gapped server) -> stored with a warning."""
    import httpx

    monkeypatch.delenv("DSTACK_SKIP_BACKEND_VALIDATION", raising=False)
    from dstack_amd.core.backends.clouds import rest_vm

    calls = []

    def fake_get(self, url, **kw):
        calls.append(url)
        req = httpx.Request("GET", url)
        if kw.get("headers", {}).get("Authorization") == "Bearer bad":
            return httpx.Response(401, text='{"error": "invalid api key"}', request=req)
        if kw.get("headers", {}).get("Authorization") == "Bearer offline":
            raise httpx.ConnectError("no route to host", request=req)
        return httpx.Response(200, json={"data": {}}, request=req)

    monkeypatch.setattr(httpx.Client, "get", fake_get)
    body = {"type": "lambda", "creds": {"type": "api_key", "api_key": "bad"}}
    r = client.post("/api/project/main/backends/create", json=body)
    assert r.status_code == 400 and r.json()["detail"][0]["code"] == "invalid_credentials", r.text
    assert calls and calls[-1].endswith("/instance-types")
    body["creds"]["api_key"] = "offline"
    r = client.post("/api/project/main/backends/create", json=body)
    assert r.status_code == 200, r.text
    # update with rejected credentials is refused too, the stored backend stays
    body["creds"]["api_key"] = "bad"
    r = client.post("/api/project/main/backends/update", json=body)
    assert r.status_code == 400
    body["creds"]["api_key"] = "good"
    assert client.post("/api/project/main/backends/update", json=body).status_code == 200


def test_credential_checks_call_each_cloud():
    """Each cloud's check_credentials hits an authenticated endpoint and maps 401/403 to an auth
    error (mock transports)."""
    import httpx

    from dstack_amd.core.backends.clouds import compute_class
    from dstack_amd.core.errors import BackendAuthError
    from dstack_amd.core.models.backends import BackendType

    seen = []

    def deny(req):
        seen.append(str(req.url))
        return httpx.Response(401 if "token" not in req.url.path else 400, text="denied")

    client = httpx.Client(transport=httpx.MockTransport(deny))
    cases = {
        BackendType.LAMBDA: ({}, {"api_key": "k"}, "/instance-types"),
        BackendType.VULTR: ({}, {"api_key": "k"}, "/account"),
        BackendType.DATACRUNCH: ({}, {"client_id": "a", "client_secret": "b"}, "/oauth2/token"),
        BackendType.CUDO: ({"project_id": "p"}, {"api_key": "k"}, "/projects/p"),
        BackendType.NEBIUS: ({"folder_id": "f"}, {"iam_token": "t"}, "/instances"),
        BackendType.VASTAI: ({}, {"api_key": "k"}, "/users/current/"),
        BackendType.RUNPOD: ({}, {"api_key": "k"}, "graphql"),
        BackendType.AWS: ({}, {"access_key": "a", "secret_key": "s"}, "sts.amazonaws.com"),
        BackendType.AZURE: ({"subscription_id": "s", "tenant_id": "t"}, {"client_id": "c", "client_secret": "x"},
                            "oauth2/v2.0/token"),
    }
    for bt, (cfg, auth, needle) in cases.items():
        c = compute_class(bt)(cfg, auth, client)
        try:
            c.check_credentials()
            raise AssertionError(f"{bt.value}: rejected credentials accepted")
        except BackendAuthError:
            pass
        assert needle in seen[-1], (bt, seen[-1])
