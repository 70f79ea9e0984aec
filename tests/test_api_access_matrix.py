"""Access control across the whole REST surface (reference: the ``test_returns_40x_if_not_authenticated``
/ ``test_returns_403_if_not_project_member`` / ``test_returns_403_if_not_admin`` cases repeated in every
``src/tests/_internal/server/routers/test_*.py``): every route of the reference server, requested

* without a token, and with an unknown token -> 401/403;
* by an authenticated user who is not a member of the project -> 403 on every project route;
* by a plain project member on the project-admin routes (backends, gateways) -> 403;
* by a non-admin on the global-admin routes (users) -> 403;

and the cross-project list endpoints return only the caller's projects."""

from __future__ import annotations

import re

import pytest

from tests.test_server_routers import REFERENCE_ROUTES

FILL = {"project_name": "main", "backend_name": "local", "run_name": "nope"}


def _url(route: str) -> str:
    return re.sub(r"\{([^}]+)\}", lambda m: FILL[m.group(1)], route)


def _method(route: str) -> str:
    return "GET" if route.endswith("/metrics/job/{run_name}") else "POST"


def _call(client, route, headers):
    url = _url(route)
    if _method(route) == "GET":
        return client.get(url, headers=headers)
    return client.post(url, json={}, headers=headers)


def _user(client, name, role="user"):
    u = client.post("/api/users/create", json={"username": name, "global_role": role}).json()
    return {"Authorization": f"Bearer {u['creds']['token']}"}


def _member(client, name, role):
    h = _user(client, name)
    members = [{"username": m["user"]["username"], "project_role": m["project_role"]}
               for m in client.post("/api/projects/main/get").json()["members"]]
    r = client.post("/api/projects/main/set_members", json={"members": members + [{"username": name,
                                                                                    "project_role": role}]})
    assert r.status_code == 200, r.text
    return h


# public in the reference too (routers/backends.py:45, routers/server.py:13)
OPEN = {"/api/backends/list_types", "/api/server/get_info"}


@pytest.mark.parametrize("route", [r for r in REFERENCE_ROUTES if r not in OPEN])
def test_every_route_requires_a_valid_token(client, route):
    """``test_returns_40x_if_not_authenticated`` of every reference router."""
    r = _call(client, route, {"Authorization": ""})
    assert r.status_code in (401, 403), (route, r.status_code, r.text[:200])
    r = _call(client, route, {"Authorization": "Bearer not-a-token"})
    assert r.status_code in (401, 403), (route, r.status_code, r.text[:200])


def test_project_routes_forbid_non_members(client):
    """``test_returns_403_if_not_project_member`` of the runs, repos, logs, metrics, fleets, volumes,
    gateways, pools, secrets and backends routers: a valid user outside the project gets 403 on every
    ``/api/project/{project}/...`` route, and cannot read the project itself."""
    outsider = _user(client, "outsider")
    project_routes = [r for r in REFERENCE_ROUTES if "{project_name}" in r]
    assert len(project_routes) > 40
    for route in project_routes:
        r = _call(client, route, outsider)
        assert r.status_code == 403, (route, r.status_code, r.text[:200])
    assert client.post("/api/projects/main/get", headers=outsider).status_code == 403
    assert client.post("/api/projects/delete", json={"projects_names": ["main"]}, headers=outsider).status_code == 403


ADMIN_ONLY = [
    "/api/project/{project_name}/backends/create",
    "/api/project/{project_name}/backends/create_yaml",
    "/api/project/{project_name}/backends/update",
    "/api/project/{project_name}/backends/update_yaml",
    "/api/project/{project_name}/backends/delete",
    "/api/project/{project_name}/backends/{backend_name}/config_info",
    "/api/project/{project_name}/backends/{backend_name}/get_yaml",
    "/api/project/{project_name}/gateways/create",
    "/api/project/{project_name}/gateways/delete",
    "/api/project/{project_name}/gateways/set_default",
    "/api/project/{project_name}/gateways/set_wildcard_domain",
]


def test_project_admin_routes_forbid_plain_members(client):
    """``test_returns_403_if_not_admin`` (backends router) and ``test_only_admin_can_*`` (gateways
    router): a project member with the ``user`` role may use the project but not administer it."""
    member = _member(client, "plain", "user")
    assert client.post("/api/project/main/fleets/list", json={}, headers=member).status_code == 200
    for route in ADMIN_ONLY:
        r = _call(client, route, member)
        assert r.status_code == 403, (route, r.status_code, r.text[:200])
    admin = _member(client, "padmin", "admin")
    # a project admin passes the role check (the empty bodies then fail validation, not auth)
    for route in ADMIN_ONLY:
        assert _call(client, route, admin).status_code != 403, route


def test_global_admin_routes(client):
    """Users router: listing, creating and deleting users and reading another user need a global
    admin; a user reads itself (``get_my_user``)."""
    u = _user(client, "reg")
    assert client.post("/api/users/create", json={"username": "x2"}, headers=u).status_code == 403
    assert client.post("/api/users/delete", json={"users": ["reg"]}, headers=u).status_code == 403
    assert client.post("/api/users/get_user", json={"username": "admin"}, headers=u).status_code in (400, 403)
    me = client.post("/api/users/get_my_user", headers=u)
    assert me.status_code == 200 and me.json()["username"] == "reg"


def test_cross_project_lists_scoped_to_the_callers_projects(client):
    """``test_non_admin_cannot_see_others_projects`` (fleets, volumes) and ``test_lists_*_across_projects``:
    the global list endpoints show a regular user only the projects they belong to, an admin all."""
    u = _user(client, "lister")
    r = client.post("/api/projects/create", json={"project_name": "listers"}, headers=u)
    assert r.status_code == 200, r.text
    for proj, name in (("main", "fm"), ("listers", "fl")):
        spec = {"spec": {"configuration": {"type": "fleet", "name": name, "nodes": 0}, "profile": {"name": "default"}}}
        hdr = None if proj == "main" else u
        assert client.post(f"/api/project/{proj}/fleets/create", json=spec, headers=hdr).status_code == 200
    mine = {f["name"] for f in client.post("/api/fleets/list", json={}, headers=u).json()}
    assert mine == {"fl"}
    everything = {f["name"] for f in client.post("/api/fleets/list", json={}).json()}
    assert {"fm", "fl"} <= everything
    assert client.post("/api/volumes/list", json={}, headers=u).json() == []
    projects = {p["project_name"] for p in client.post("/api/projects/list", headers=u).json()}
    assert projects == {"listers"}
    runs = client.post("/api/runs/list", json={}, headers=u).json()
    assert all(r["project_name"] == "listers" for r in runs)
    insts = client.post("/api/instances/list", json={}, headers=u).json()
    assert all(i["project_name"] == "listers" for i in insts)
