"""Users, projects/members and logs APIs (reference: ``src/tests/_internal/server/routers/test_{users,
projects,logs}.py``): role checks, project quotas, managers cannot touch admins, deleted/inactive
users lose access, token refresh; log polling windows (exclusive bounds), limits, descending order
and ``next_token`` paging in both directions, runner (diagnose) logs."""

from __future__ import annotations

import base64
import uuid
from datetime import datetime, timedelta, timezone

import pytest

from dstack_amd.server.services import logs as logs_services


def _user(client, name, role="user"):
    r = client.post("/api/users/create", json={"username": name, "global_role": role})
    assert r.status_code == 200, r.text
    return {"Authorization": f"Bearer {r.json()['creds']['token']}"}


def _members(client, project, members, headers=None):
    return client.post(f"/api/projects/{project}/set_members", headers=headers,
                       json={"members": [{"username": u, "project_role": r} for u, r in members]})


# ---- users --------------------------------------------------------------------------------------
def test_user_update_and_inactive_user_locked_out(client):
    h = _user(client, "ivan")
    assert client.post("/api/users/get_my_user", headers=h).status_code == 200
    r = client.post("/api/users/update", json={"username": "ivan", "global_role": "admin", "email": "i@x"})
    assert r.status_code == 200 and r.json()["global_role"] == "admin"
    assert client.post("/api/users/create", json={"username": "by-ivan"}, headers=h).status_code == 200
    client.post("/api/users/update", json={"username": "ivan", "global_role": "user", "active": False})
    assert client.post("/api/users/get_my_user", headers=h).status_code in (401, 403)


def test_get_user_and_refresh_token_rules(client):
    a = _user(client, "ann")
    _user(client, "ben")
    assert client.post("/api/users/get_user", json={"username": "ann"}, headers=a).status_code == 200
    assert client.post("/api/users/get_user", json={"username": "ben"}, headers=a).status_code == 403
    assert client.post("/api/users/refresh_token", json={"username": "ben"}, headers=a).status_code == 403
    new = client.post("/api/users/refresh_token", json={"username": "ann"}, headers=a).json()["creds"]["token"]
    assert client.post("/api/users/get_my_user", headers=a).status_code in (401, 403)  # old token revoked
    assert client.post("/api/users/get_my_user", headers={"Authorization": f"Bearer {new}"}).status_code == 200


def test_deleted_user_loses_access(client):
    h = _user(client, "gone")
    client.post("/api/users/delete", json={"users": ["gone"]})
    assert client.post("/api/users/get_my_user", headers=h).status_code in (401, 403)


# ---- projects -------------------------------------------------------------------------------------
def test_project_quota_for_regular_users(client, monkeypatch):
    from dstack_amd.server import settings

    monkeypatch.setattr(settings, "USER_PROJECT_DEFAULT_QUOTA", 3)  # DSTACK_USER_PROJECT_DEFAULT_QUOTA
    h = _user(client, "quota")
    for i in range(3):
        assert client.post("/api/projects/create", json={"project_name": f"q{i}"}, headers=h).status_code == 200
    r = client.post("/api/projects/create", json={"project_name": "q3"}, headers=h)
    assert r.status_code == 400 and "quota" in r.text
    for i in range(5):  # global admins have no quota
        assert client.post("/api/projects/create", json={"project_name": f"admin{i}"}).status_code == 200


def test_project_creator_is_admin_and_can_delete(client):
    h = _user(client, "owner")
    client.post("/api/projects/create", json={"project_name": "mine"}, headers=h)
    client.post("/api/projects/create", json={"project_name": "spare"}, headers=h)  # not the only one
    got = client.post("/api/projects/mine/get", headers=h).json()
    assert [(m["user"]["username"], m["project_role"]) for m in got["members"]] == [("owner", "admin")]
    other = _user(client, "other")
    assert client.post("/api/projects/delete", json={"projects_names": ["mine"]}, headers=other).status_code == 403
    assert client.post("/api/projects/delete", json={"projects_names": ["mine"]}, headers=h).status_code == 200
    assert client.post("/api/projects/mine/get", headers=h).status_code in (400, 403, 404)
    # the name is free again
    assert client.post("/api/projects/create", json={"project_name": "mine"}, headers=h).status_code == 200


def test_manager_manages_users_but_not_admins(client):
    mgr = _user(client, "mgr")
    _user(client, "dev")
    _user(client, "boss")
    assert _members(client, "main", [("admin", "admin"), ("mgr", "manager")]).status_code == 200
    # a manager adds a user
    assert _members(client, "main", [("admin", "admin"), ("mgr", "manager"), ("dev", "user")],
                    headers=mgr).status_code == 200
    # ... but cannot add or remove admins
    r = _members(client, "main", [("admin", "admin"), ("boss", "admin"), ("mgr", "manager")], headers=mgr)
    assert r.status_code == 403
    assert _members(client, "main", [("mgr", "manager")], headers=mgr).status_code == 403
    # a plain user cannot manage members at all
    dev = client.post("/api/users/refresh_token", json={"username": "dev"}).json()["creds"]["token"]
    assert _members(client, "main", [("admin", "admin")], headers={"Authorization": f"Bearer {dev}"}).status_code == 403


def test_project_roles_gate_backends_and_secrets(client):
    mgr = _user(client, "m2")
    usr = _user(client, "u2")
    _members(client, "main", [("admin", "admin"), ("m2", "manager"), ("u2", "user")])
    vultr = {"type": "vultr", "creds": {"type": "api_key", "api_key": "k"}}
    assert client.post("/api/project/main/backends/create", json=vultr, headers=mgr).status_code == 403
    assert client.post("/api/project/main/secrets/add", json={"name": "A", "value": "1"}, headers=mgr).status_code == 200
    assert client.post("/api/project/main/secrets/list", headers=usr).status_code == 403
    assert client.post("/api/project/main/fleets/list", headers=usr).status_code == 200


# ---- logs -----------------------------------------------------------------------------------------
T0 = datetime(2026, 1, 1, tzinfo=timezone.utc)


def _write(sub: str, n: int, run="logrun"):
    events = [{"timestamp": int((T0 + timedelta(seconds=i)).timestamp() * 1000),
               "message": base64.b64encode(f"line {i}\n".encode()).decode()} for i in range(n)]
    logs_services.get_default_log_storage().write_logs("main", run, sub, [{"timestamp": events[0]["timestamp"],
                                                                            "message": base64.b64encode(b"runner\n")
                                                                            .decode()}], events)


def _poll(client, sub, **kw):
    body = {"run_name": "logrun", "job_submission_id": sub, **kw}
    r = client.post("/api/project/main/logs/poll", json=body)
    assert r.status_code == 200, r.text
    d = r.json()
    return [base64.b64decode(e["message"]).decode().strip() for e in d["logs"]], d.get("next_token")


def test_logs_window_limit_and_paging(client):
    sub = str(uuid.uuid4())
    _write(sub, 10)
    lines, tok = _poll(client, sub)
    assert lines == [f"line {i}" for i in range(10)] and tok is None
    # exclusive bounds
    lines, _ = _poll(client, sub, start_time=(T0 + timedelta(seconds=2)).isoformat(),
                     end_time=(T0 + timedelta(seconds=5)).isoformat())
    assert lines == ["line 3", "line 4"]
    # forward pages of 4
    seen, tok = [], None
    while True:
        kw = {"limit": 4}
        if tok:
            kw["next_token"] = tok
        lines, tok = _poll(client, sub, **kw)
        seen += lines
        if not tok:
            break
    assert seen == [f"line {i}" for i in range(10)]
    # backward pages of 4, newest first
    seen, tok = [], None
    while True:
        kw = {"limit": 4, "descending": True}
        if tok:
            kw["next_token"] = tok
        lines, tok = _poll(client, sub, **kw)
        seen += lines
        if not tok:
            break
    assert seen == [f"line {i}" for i in reversed(range(10))]


def test_runner_logs_with_diagnose(client):
    sub = str(uuid.uuid4())
    _write(sub, 2)
    lines, _ = _poll(client, sub, diagnose=True)
    assert lines == ["runner"]


def test_logs_appended_across_pulls_are_indexed(client):
    sub = str(uuid.uuid4())
    _write(sub, 3)
    assert len(_poll(client, sub)[0]) == 3
    storage = logs_services.get_default_log_storage()
    later = [{"timestamp": int((T0 + timedelta(seconds=10 + i)).timestamp() * 1000),
              "message": base64.b64encode(f"late {i}\n".encode()).decode()} for i in range(2)]
    storage.write_logs("main", "logrun", sub, [], later)
    lines, _ = _poll(client, sub, start_time=(T0 + timedelta(seconds=2)).isoformat())
    assert lines == ["late 0", "late 1"]


@pytest.mark.parametrize("bad", ["not-a-date", "2026-13-01"])
def test_bad_next_token(client, bad):
    r = client.post("/api/project/main/logs/poll", json={"run_name": "x", "job_submission_id": str(uuid.uuid4()),
                                                         "next_token": bad})
    assert r.status_code == 400
