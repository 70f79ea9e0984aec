"""Gateway control API, nginx sites, stats and the OpenAI model proxy, case by case against the
reference's ``src/tests/_internal/proxy/{gateway,lib}`` (mapping: ``docs/reference/test-parity.md``).
nginx, certbot and ``nginx -t`` are stand-in commands; a replica is a local HTTP server or, for the
connection failure, an SSH forward to a closed port."""

from __future__ import annotations

import json
import socket
import time

import pytest
from fastapi.testclient import TestClient

from dstack_amd.proxy.gateway.app import Gateway, make_app
from dstack_amd.proxy.gateway.nginx import Nginx
from dstack_amd.proxy.gateway.registry import Registry
from dstack_amd.proxy.gateway.stats import StatsCollector
from tests.test_gateway import upstream  # noqa: F401  (fixture: a local HTTP replica)


@pytest.fixture
def gw(tmp_path):
    ng = Nginx(conf_dir=str(tmp_path / "sites"), access_log=str(tmp_path / "access.log"), reload_cmd=["true"],
               test_cmd=["true"], certbot_cmd=["true"], certs_dir=str(tmp_path / "certs"))
    g = Gateway(tmp_path / "state", nginx=ng)
    g.conns.connect_timeout = 5.0
    return g


def _site(gw, domain):
    p = gw.nginx.conf_dir / gw.nginx.site_name(domain)
    return p.read_text() if p.exists() else None


def _svc(c, project="main", run="svc", **kw):
    body = {"run_name": run, "domain": f"{run}.{project}.example.com", "auth": False, **kw}
    return c.post(f"/api/registry/{project}/services/register", json=body)


def _rep(c, port, project="main", run="svc", job="job-0", **kw):
    return c.post(f"/api/registry/{project}/services/{run}/replicas/register",
                  json={"job_id": job, "app_port": port, "internal_ip": "127.0.0.1", **kw})


# ---- routers/test_registry.py: services ----------------------------------------------------------
def test_register_service(gw):
    c = TestClient(make_app(gw))
    assert _svc(c).status_code == 200
    site = _site(gw, "svc.main.example.com")
    assert "server_name svc.main.example.com;" in site and "listen 80;" in site
    assert "return 503;" in site and "auth_request" not in site and "ssl" not in site  # no replicas yet
    assert gw.registry.get_service("main", "svc") is not None


def test_register_service_with_https(gw):
    c = TestClient(make_app(gw))
    assert _svc(c, https=True).status_code == 200
    site = _site(gw, "svc.main.example.com")
    assert "listen 443 ssl;" in site and f"{gw.nginx.certs_dir}/svc.main.example.com/fullchain.pem" in site
    assert "return 301 https://$host$request_uri;" in site


def test_register_service_with_auth(gw):
    c = TestClient(make_app(gw))
    assert _svc(c, auth=True).status_code == 200
    site = _site(gw, "svc.main.example.com")
    assert "auth_request /_dstack_auth;" in site and "/api/auth/main;" in site


def test_register_same_name_error(gw):
    c = TestClient(make_app(gw))
    assert _svc(c).status_code == 200
    r = _svc(c)
    assert r.status_code == 400 and "already registered" in r.json()["detail"]


def test_register_same_name_in_different_projects(gw):
    c = TestClient(make_app(gw))
    assert _svc(c, project="p1").status_code == 200 and _svc(c, project="p2").status_code == 200
    assert {s.key for s in gw.registry.services.values()} == {"p1/svc", "p2/svc"}
    assert _site(gw, "svc.p1.example.com") and _site(gw, "svc.p2.example.com")


def test_register_service_with_model(gw):
    c = TestClient(make_app(gw))
    r = _svc(c, options={"openai": {"model": {"name": "llama", "format": "openai", "prefix": "/v1"}}})
    assert r.status_code == 200
    assert [m["id"] for m in c.get("/api/models/main/models").json()["data"]] == ["llama"]


# ---- routers/test_registry.py: replicas ----------------------------------------------------------
def test_register_replica(gw, upstream):  # noqa: F811
    c = TestClient(make_app(gw))
    _svc(c)
    assert _rep(c, upstream).status_code == 200
    site = _site(gw, "svc.main.example.com")
    assert f"server 127.0.0.1:{upstream};" in site and "proxy_pass http://dstack_main_svc;" in site


def test_register_replica_no_service_error(gw):
    c = TestClient(make_app(gw))
    r = _rep(c, 8000)
    assert r.status_code == 400 and "not registered" in r.json()["detail"]


def test_register_replica_twice_error(gw, upstream):  # noqa: F811
    c = TestClient(make_app(gw))
    _svc(c)
    assert _rep(c, upstream).status_code == 200
    r = _rep(c, upstream)
    assert r.status_code == 400 and "already registered" in r.json()["detail"]
    assert len(gw.registry.get_service("main", "svc").replicas) == 1


def test_register_replica_connection_error(gw):
    """A replica behind SSH whose forward cannot be set up is refused and not routed to."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        closed_port = s.getsockname()[1]  # bound, then released: nothing listens here
    c = TestClient(make_app(gw))
    _svc(c)
    r = _rep(c, 8000, ssh_host="nobody@127.0.0.1", ssh_port=closed_port, direct=False)
    assert r.status_code == 400 and "cannot connect to replica" in r.json()["detail"]
    assert gw.registry.get_service("main", "svc").replicas == {}
    assert "return 503;" in _site(gw, "svc.main.example.com")


# ---- routers/test_registry.py: unregister ---------------------------------------------------------
def test_unregister_service(gw):
    c = TestClient(make_app(gw))
    _svc(c)
    assert c.post("/api/registry/main/services/svc/unregister").status_code == 200
    assert gw.registry.get_service("main", "svc") is None and _site(gw, "svc.main.example.com") is None


def test_unregister_service_not_registered_error(gw):
    c = TestClient(make_app(gw))
    r = c.post("/api/registry/main/services/svc/unregister")
    assert r.status_code == 400 and "not registered" in r.json()["detail"]


def test_unregister_service_with_replicas(gw, upstream):  # noqa: F811
    c = TestClient(make_app(gw))
    _svc(c)
    _rep(c, upstream, job="a")
    _rep(c, upstream, job="b")
    closed = []
    gw.conns.close = closed.append
    assert c.post("/api/registry/main/services/svc/unregister").status_code == 200
    assert sorted(closed) == ["a", "b"] and _site(gw, "svc.main.example.com") is None


def test_unregister_service_with_model(gw):
    c = TestClient(make_app(gw))
    _svc(c, options={"openai": {"model": {"name": "llama", "format": "openai"}}})
    c.post("/api/registry/main/services/svc/unregister")
    assert c.get("/api/models/main/models").json()["data"] == []


def test_unregister_replica(gw, upstream):  # noqa: F811
    c = TestClient(make_app(gw))
    _svc(c)
    _rep(c, upstream)
    assert c.post("/api/registry/main/services/svc/replicas/job-0/unregister").status_code == 200
    assert gw.registry.get_service("main", "svc").replicas == {}
    assert "return 503;" in _site(gw, "svc.main.example.com")


def test_unregister_replica_no_replica_error(gw):
    c = TestClient(make_app(gw))
    _svc(c)
    r = c.post("/api/registry/main/services/svc/replicas/job-0/unregister")
    assert r.status_code == 400 and "not registered" in r.json()["detail"]


def test_unregister_replica_no_service_error(gw):
    c = TestClient(make_app(gw))
    r = c.post("/api/registry/main/services/svc/replicas/job-0/unregister")
    assert r.status_code == 400 and "not registered" in r.json()["detail"]


# ---- routers/test_registry.py: entrypoints ---------------------------------------------------------
@pytest.mark.parametrize("https", [False, True])
def test_register_entrypoint(gw, https):
    c = TestClient(make_app(gw))
    r = c.post("/api/registry/main/entrypoints/register", json={"domain": "gateway.example.com", "https": https})
    assert r.status_code == 200
    site = _site(gw, "gateway.example.com")
    assert "server_name gateway.example.com;" in site and "/api/models/main/;" in site
    assert ("listen 443 ssl;" in site) is https


# ---- routers/test_stats.py, services/test_stats.py ------------------------------------------------
def test_collect_stats_per_service(gw):
    c = TestClient(make_app(gw))
    _svc(c, run="a")
    _svc(c, run="b")
    now = time.time()
    for i in range(4):
        gw.stats.record("a.main.example.com", 0.5, now - i)
    out = {x["run_name"]: x["stats"] for x in c.get("/api/stats/collect").json()}
    assert out["a"]["30"] == {"requests": 4, "request_time": 0.5}
    assert out["b"]["300"] == {"requests": 0, "request_time": 0.0}


def test_collect_stats_from_access_log_and_after_update(tmp_path):
    log = tmp_path / "access.log"
    now = time.time()
    log.write_text("".join(f"{now - 40 - i:.3f} svc.example.com 200 0.2\n" for i in range(3)) +
                   f"{now - 1:.3f} svc.example.com 200 0.4\n{now - 1:.3f} other.example.com 502 1.0\n")
    sc = StatsCollector(str(log))
    st = sc.collect()
    assert st["svc.example.com"][30]["requests"] == 1 and st["svc.example.com"][60]["requests"] == 4
    assert abs(st["svc.example.com"][60]["request_time"] - 0.25) < 1e-9
    with open(log, "a") as f:  # new lines after the first read are picked up incrementally
        f.write(f"{time.time():.3f} svc.example.com 200 0.6\npartial-line-without-newline")
    st = sc.collect()
    assert st["svc.example.com"][30]["requests"] == 2


# ---- test_app.py, repo/test_repo.py, repo/test_state_v1.py ----------------------------------------
def test_lifespan_restores_state_and_closes_on_shutdown(tmp_path, upstream):  # noqa: F811
    ng = lambda: Nginx(conf_dir=str(tmp_path / "sites"), access_log=str(tmp_path / "a.log"),  # noqa: E731
                       reload_cmd=["true"], test_cmd=["true"], certbot_cmd=["true"])
    g1 = Gateway(tmp_path / "state", nginx=ng())
    with TestClient(make_app(g1)) as c:
        _svc(c)
        _rep(c, upstream)
    assert g1.http.is_closed  # shutdown closed the upstream client
    (tmp_path / "sites" / "80-svc.main.example.com.conf").unlink()
    g2 = Gateway(tmp_path / "state", nginx=ng())  # a restarted gateway re-renders its sites
    assert g2.registry.get_service("main", "svc").replicas["job-0"].app_port == upstream
    assert f"127.0.0.1:{upstream}" in (tmp_path / "sites" / "80-svc.main.example.com.conf").read_text()


def test_persist_repo(tmp_path):
    from dstack_amd.proxy.gateway.registry import Replica

    r = Registry(tmp_path / "s.json")
    r.register_service("p", "svc", "svc.example.com", https=True, auth=False,
                       model={"name": "m", "format": "openai"})
    r.add_replica("p", "svc", Replica(id="j", app_port=8000, internal_ip="10.0.0.2"))
    r.register_entrypoint("p", "gateway.example.com", https=True)
    r.acme["server_url"] = "http://server:3000"
    r.save()
    again = Registry(tmp_path / "s.json")
    svc = again.get_service("p", "svc")
    assert (svc.https, svc.auth, svc.model["name"], svc.replicas["j"].upstream()) == (True, False, "m", "10.0.0.2:8000")
    assert again.entrypoints["p"].https and again.acme == {"server_url": "http://server:3000"}
    assert json.loads((tmp_path / "s.json").read_text())["version"] == 2


# ---- lib/routers/test_model_proxy.py --------------------------------------------------------------
def _model_svc(c, port, run="llm", auth=False):
    _svc(c, run=run, auth=auth, options={"openai": {"model": {"name": "llama", "format": "openai", "prefix": "/v1"}}})
    _rep(c, port, run=run)


def test_model_proxy_list_models(gw, upstream):  # noqa: F811
    c = TestClient(make_app(gw))
    _model_svc(c, upstream)
    data = c.get("/api/models/main/models").json()
    assert data["object"] == "list" and [(m["id"], m["object"]) for m in data["data"]] == [("llama", "model")]


def test_model_proxy_list_models_empty(gw):
    c = TestClient(make_app(gw))
    assert c.get("/api/models/main/models").json() == {"object": "list", "data": []}


def test_model_proxy_chat_completions(gw, upstream):  # noqa: F811
    c = TestClient(make_app(gw))
    _model_svc(c, upstream)
    r = c.post("/api/models/main/chat/completions", json={"model": "llama", "messages": [{"role": "user", "content": "ping"}]})
    assert r.status_code == 200 and r.json()["choices"][0]["message"]["content"] == "pong"


def test_model_proxy_chat_completions_model_not_found(gw):
    c = TestClient(make_app(gw))
    r = c.post("/api/models/main/chat/completions", json={"model": "nope", "messages": []})
    assert r.status_code == 404 and "not found" in r.json()["detail"]


@pytest.mark.parametrize("token,status", [("good", 200), ("bad", 403), (None, 403)])
def test_model_proxy_auth(gw, upstream, monkeypatch, token, status):  # noqa: F811
    async def member(project, tok):
        return tok == "good"

    monkeypatch.setattr(gw.auth, "is_member", member)
    c = TestClient(make_app(gw))
    _model_svc(c, upstream, auth=True)
    headers = {"Authorization": f"Bearer {token}"} if token else {}
    r = c.post("/api/models/main/chat/completions", headers=headers,
               json={"model": "llama", "messages": [{"role": "user", "content": "ping"}]})
    assert r.status_code == status


class _SSEHandler(__import__("http.server").server.BaseHTTPRequestHandler):
    """An OpenAI-format replica streaming three chunks and a TGI one streaming tokens."""

    protocol_version = "HTTP/1.1"

    def do_POST(self):
        req = json.loads(self.rfile.read(int(self.headers.get("content-length", 0))) or b"{}")
        if self.path == "/v1/chat/completions":
            events = [json.dumps({"object": "chat.completion.chunk", "model": req["model"],
                                  "choices": [{"index": 0, "delta": {"content": t}, "finish_reason": None}]})
                      for t in ("po", "n", "g")] + ["[DONE]"]
        else:  # TGI /generate_stream
            toks = [("po", None), ("ng", None), ("<|eot_id|>", {"finish_reason": "eos_token"})]
            events = [json.dumps({"token": {"text": t}, "details": d}) for t, d in toks]
        body = "".join(f"data: {e}\n\n" for e in events).encode()
        self.send_response(200)
        self.send_header("content-type", "text/event-stream")
        self.send_header("content-length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def log_message(self, *a):
        pass


def test_model_proxy_chat_completions_stream(gw):
    import http.server
    import threading

    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), _SSEHandler)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        c = TestClient(make_app(gw))
        _model_svc(c, srv.server_address[1])
        _svc(c, run="tgi", options={"openai": {"model": {"name": "llama-tgi", "format": "tgi"}}})
        _rep(c, srv.server_address[1], run="tgi")
        for model in ("llama", "llama-tgi"):
            with c.stream("POST", "/api/models/main/chat/completions",
                          json={"model": model, "stream": True, "messages": [{"role": "user", "content": "ping"}]}) as r:
                assert r.status_code == 200 and r.headers["content-type"].startswith("text/event-stream")
                events = [ln[6:] for ln in r.iter_lines() if ln.startswith("data: ")]
            assert events[-1] == "[DONE]"
            chunks = [json.loads(e) for e in events[:-1]]
            assert "".join(ch["choices"][0]["delta"].get("content", "") for ch in chunks) == "pong"
            assert all(ch["object"] == "chat.completion.chunk" for ch in chunks)
    finally:
        srv.shutdown()
