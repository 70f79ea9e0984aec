"""Users and projects routers, case by case against the reference's ``routers/test_users.py`` and
``routers/test_projects.py`` (mapping: ``docs/reference/test-parity.md``).  The unauthenticated /
non-member cases of both routers are in ``test_api_access_matrix.py``."""

from __future__ import annotations

from tests.conftest import ADMIN_TOKEN


def _user(client, name, role="user"):
    r = client.post("/api/users/create", json={"username": name, "global_role": role})
    assert r.status_code == 200, r.text
    return r.json(), {"Authorization": f"Bearer {r.json()['creds']['token']}"}


def _members(client, project, *pairs, headers=None):
    return client.post(f"/api/projects/{project}/set_members", headers=headers,
                       json={"members": [{"username": u, "project_role": r} for u, r in pairs]})


# ---- users ------------------------------------------------------------------------------------
def test_list_users_admin_sees_everyone_user_sees_self(client):
    _user(client, "u1")
    _, h2 = _user(client, "u2")
    names = {u["username"] for u in client.post("/api/users/list").json()}
    assert {"admin", "u1", "u2"} <= names
    assert [u["username"] for u in client.post("/api/users/list", headers=h2).json()] == ["u2"]


def test_get_my_user_returns_logged_in_user_with_token(client):
    me = client.post("/api/users/get_my_user").json()
    assert me["username"] == "admin" and me["global_role"] == "admin" and me["creds"]["token"] == ADMIN_TOKEN


def test_get_my_user_rejects_deactivated_user(client):
    _, h = _user(client, "gone")
    assert client.post("/api/users/update", json={"username": "gone", "global_role": "user", "active": False}
                       ).status_code == 200
    assert client.post("/api/users/get_my_user", headers=h).status_code in (401, 403)


def test_get_user_admin_reads_anyone_user_reads_only_self(client):
    _user(client, "alice")
    _, hb = _user(client, "bob")
    got = client.post("/api/users/get_user", json={"username": "alice"})
    assert got.status_code == 200 and got.json()["username"] == "alice" and got.json()["creds"]["token"]
    assert client.post("/api/users/get_user", json={"username": "alice"}, headers=hb).status_code in (400, 403)
    assert client.post("/api/users/get_user", json={"username": "bob"}, headers=hb).json()["username"] == "bob"
    assert client.post("/api/users/get_user", json={"username": "nobody"}).status_code == 400


def test_create_user_returns_user_with_token(client):
    u, h = _user(client, "carol", role="admin")
    assert u["username"] == "carol" and u["global_role"] == "admin" and len(u["creds"]["token"]) >= 16
    assert client.post("/api/users/get_my_user", headers=h).json()["username"] == "carol"


def test_create_user_rejects_taken_username(client):
    _user(client, "dave")
    r = client.post("/api/users/create", json={"username": "dave", "global_role": "user"})
    assert r.status_code == 400 and "exist" in r.text.lower()


def test_delete_users_revokes_access(client):
    _, h = _user(client, "erin")
    assert client.post("/api/users/delete", json={"users": ["erin"]}).status_code == 200
    assert "erin" not in {u["username"] for u in client.post("/api/users/list").json()}
    assert client.post("/api/users/get_my_user", headers=h).status_code in (401, 403)


def test_refresh_token_replaces_own_token(client):
    u, h = _user(client, "frank")
    r = client.post("/api/users/refresh_token", json={"username": "frank"}, headers=h)
    assert r.status_code == 200
    new = r.json()["creds"]["token"]
    assert new != u["creds"]["token"]
    assert client.post("/api/users/get_my_user", headers=h).status_code in (401, 403)
    assert client.post("/api/users/get_my_user", headers={"Authorization": f"Bearer {new}"}).status_code == 200


def test_refresh_token_for_another_user_needs_global_admin(client):
    _user(client, "gina")
    _, hh = _user(client, "hank")
    assert client.post("/api/users/refresh_token", json={"username": "gina"}, headers=hh).status_code == 403
    r = client.post("/api/users/refresh_token", json={"username": "gina"})
    assert r.status_code == 200 and r.json()["username"] == "gina"


# ---- projects ---------------------------------------------------------------------------------
def test_list_projects_empty_for_a_user_without_projects(client):
    _, h = _user(client, "nobody")
    assert client.post("/api/projects/list", headers=h).json() == []


def test_list_projects_returns_member_projects(client):
    projects = client.post("/api/projects/list").json()
    assert [p["project_name"] for p in projects] == ["main"]
    assert projects[0]["owner"]["username"] == "admin"
    assert {m["user"]["username"] for m in projects[0]["members"]} == {"admin"}


def test_create_project_creator_is_admin_member(client):
    _, h = _user(client, "ivy")
    r = client.post("/api/projects/create", json={"project_name": "ivyproj"}, headers=h)
    assert r.status_code == 200, r.text
    p = r.json()
    assert p["project_name"] == "ivyproj" and p["owner"]["username"] == "ivy"
    assert [(m["user"]["username"], m["project_role"]) for m in p["members"]] == [("ivy", "admin")]


def test_create_project_rejects_taken_name(client):
    r = client.post("/api/projects/create", json={"project_name": "main"})
    assert r.status_code == 400 and "exist" in r.text.lower()


def test_create_project_user_quota(client, monkeypatch):
    from dstack_amd.server import settings

    monkeypatch.setattr(settings, "USER_PROJECT_DEFAULT_QUOTA", 1)
    _, h = _user(client, "quota")
    assert client.post("/api/projects/create", json={"project_name": "q1"}, headers=h).status_code == 200
    r = client.post("/api/projects/create", json={"project_name": "q2"}, headers=h)
    assert r.status_code == 400 and "quota" in r.text.lower()
    # global admins have no quota
    for i in range(3):
        assert client.post("/api/projects/create", json={"project_name": f"adm{i}"}).status_code == 200


def test_delete_project_rules(client):
    _, hu = _user(client, "jack")
    assert client.post("/api/projects/create", json={"project_name": "jp"}, headers=hu).status_code == 200
    # a regular user cannot delete the only project they have
    r = client.post("/api/projects/delete", json={"projects_names": ["jp"]}, headers=hu)
    assert r.status_code == 400 and "only project" in r.text
    assert client.post("/api/projects/create", json={"project_name": "jp2"}, headers=hu).status_code == 200
    _, hm = _user(client, "kate")
    # a member who is not a project admin cannot delete it
    assert _members(client, "jp", ("jack", "admin"), ("kate", "user"), headers=hu).status_code == 200
    assert client.post("/api/projects/delete", json={"projects_names": ["jp"]}, headers=hm).status_code == 403
    assert client.post("/api/projects/delete", json={"projects_names": ["jp"]}, headers=hu).status_code == 200
    assert "jp" not in {p["project_name"] for p in client.post("/api/projects/list").json()}


def test_get_project(client):
    assert client.post("/api/projects/nope/get").status_code in (400, 404)
    p = client.post("/api/projects/main/get").json()
    assert p["project_name"] == "main" and p["backends"] is not None


def test_set_project_members(client):
    _user(client, "m1")
    _user(client, "m2")
    r = _members(client, "main", ("admin", "admin"), ("m1", "manager"), ("m2", "user"))
    assert r.status_code == 200, r.text
    roles = {m["user"]["username"]: m["project_role"] for m in r.json()["members"]}
    assert roles == {"admin": "admin", "m1": "manager", "m2": "user"}


def test_manager_cannot_set_project_admins(client):
    _, hm = _user(client, "mgr")
    _user(client, "other")
    assert _members(client, "main", ("admin", "admin"), ("mgr", "manager")).status_code == 200
    r = _members(client, "main", ("admin", "admin"), ("mgr", "manager"), ("other", "admin"), headers=hm)
    assert r.status_code == 403
    r = _members(client, "main", ("admin", "admin"), ("mgr", "manager"), ("other", "user"), headers=hm)
    assert r.status_code == 200, r.text


def test_global_admin_manager_can_set_project_admins(client):
    _, hg = _user(client, "gadmin", role="admin")
    _user(client, "promoted")
    assert _members(client, "main", ("admin", "admin"), ("gadmin", "manager")).status_code == 200
    r = _members(client, "main", ("admin", "admin"), ("gadmin", "manager"), ("promoted", "admin"), headers=hg)
    assert r.status_code == 200, r.text
    assert {m["user"]["username"]: m["project_role"] for m in r.json()["members"]}["promoted"] == "admin"


def test_non_manager_cannot_set_project_members(client):
    _, hu = _user(client, "plainuser")
    assert _members(client, "main", ("admin", "admin"), ("plainuser", "user")).status_code == 200
    r = _members(client, "main", ("admin", "admin"), ("plainuser", "admin"), headers=hu)
    assert r.status_code == 403
