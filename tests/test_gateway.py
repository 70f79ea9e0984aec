"""Gateway tests (reference: ``src/tests/_internal/proxy/gateway/{test_app,routers/test_registry,
routers/test_stats,services/test_stats,repo/test_repo}.py``, ``proxy/lib/routers/test_model_proxy.py``)."""

import http.server
import json
import threading
import time

import pytest
from fastapi.testclient import TestClient

from dstack_amd.proxy.gateway.app import Gateway, make_app, make_dataplane_app
from dstack_amd.proxy.gateway.nginx import Nginx
from dstack_amd.proxy.gateway.registry import Registry, RegistryError, Replica
from dstack_amd.proxy.gateway.stats import StatsCollector


class _Handler(http.server.BaseHTTPRequestHandler):
    def do_GET(self):
        body = json.dumps({"path": self.path, "host": self.headers.get("host")}).encode()
        self.send_response(200)
        self.send_header("content-type", "application/json")
        self.send_header("content-length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def do_POST(self):
        n = int(self.headers.get("content-length", 0))
        req = json.loads(self.rfile.read(n) or b"{}")
        if self.path == "/v1/chat/completions":
            out = {"id": "x", "object": "chat.completion", "model": req["model"],
                   "choices": [{"index": 0, "message": {"role": "assistant", "content": "pong"},
                                "finish_reason": "stop"}]}
        elif self.path == "/generate":  # TGI
            out = {"generated_text": "tgi-answer<|eot_id|>", "details": {"finish_reason": "eos_token",
                                                                         "generated_tokens": 3}}
        else:
            out = {"echo": req}
        body = json.dumps(out).encode()
        self.send_response(200)
        self.send_header("content-type", "application/json")
        self.send_header("content-length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def log_message(self, *a):
        pass


@pytest.fixture
def upstream():
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), _Handler)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    yield srv.server_address[1]
    srv.shutdown()


@pytest.fixture
def gw(tmp_path):
    return Gateway(tmp_path)


def _register(c, upstream_port, run="svc", auth=False, model=None):
    opts = {"openai": {"model": model}} if model else {}
    r = c.post("/api/registry/main/services/register",
               json={"run_name": run, "domain": f"{run}.example.com", "auth": auth, "options": opts})
    assert r.status_code == 200, r.text
    r = c.post(f"/api/registry/main/services/{run}/replicas/register",
               json={"job_id": f"{run}-job0", "app_port": upstream_port, "internal_ip": "127.0.0.1"})
    assert r.status_code == 200, r.text


def test_registry_lifecycle_and_persistence(tmp_path):
    reg = Registry(tmp_path / "state.json")
    reg.register_service("p", "a", "a.example.com")
    with pytest.raises(RegistryError):
        reg.register_service("p", "a", "a2.example.com")
    with pytest.raises(RegistryError):
        reg.register_service("p", "b", "a.example.com")  # domain taken
    reg.add_replica("p", "a", Replica(id="j1", app_port=8000, internal_ip="10.0.0.5"))
    reg.register_entrypoint("p", "gateway.example.com")
    again = Registry(tmp_path / "state.json")
    svc = again.get_service("p", "a")
    assert svc is not None and svc.replicas["j1"].upstream() == "10.0.0.5:8000"
    assert again.entrypoint_by_domain("GATEWAY.example.com:443").project == "p"
    again.remove_replica("p", "a", "j1")
    again.unregister_service("p", "a")
    assert Registry(tmp_path / "state.json").services == {}


def test_dataplane_routes_by_host_and_round_robins(gw, upstream):
    ctl = TestClient(make_app(gw))
    _register(ctl, upstream)
    dp = TestClient(make_dataplane_app(gw))
    r = dp.get("/hello?x=1", headers={"host": "svc.example.com"})
    assert r.status_code == 200
    assert r.json()["path"] == "/hello?x=1"
    assert dp.get("/", headers={"host": "unknown.example.com"}).status_code == 404
    # unregister the only replica -> 503
    ctl.post("/api/registry/main/services/svc/replicas/svc-job0/unregister")
    assert dp.get("/", headers={"host": "svc.example.com"}).status_code == 503


def test_dataplane_auth(gw, upstream, monkeypatch):
    ctl = TestClient(make_app(gw))
    _register(ctl, upstream, run="private", auth=True)
    dp = TestClient(make_dataplane_app(gw))
    assert dp.get("/", headers={"host": "private.example.com"}).status_code == 403

    async def fake_member(project, token):
        return token == "good"

    monkeypatch.setattr(gw.auth, "is_member", fake_member)
    assert dp.get("/", headers={"host": "private.example.com", "authorization": "Bearer bad"}).status_code == 403
    assert dp.get("/", headers={"host": "private.example.com", "authorization": "Bearer good"}).status_code == 200
    assert ctl.get("/api/auth/main", headers={"authorization": "Bearer good"}).status_code == 200


def test_stats_collect(gw, upstream):
    ctl = TestClient(make_app(gw))
    _register(ctl, upstream)
    dp = TestClient(make_dataplane_app(gw))
    for _ in range(5):
        dp.get("/", headers={"host": "svc.example.com"})
    stats = ctl.get("/api/stats/collect").json()
    s = next(x for x in stats if x["run_name"] == "svc")
    assert s["stats"]["30"]["requests"] == 5
    assert s["stats"]["300"]["request_time"] > 0


def test_stats_from_access_log(tmp_path):
    log = tmp_path / "access.log"
    now = time.time()
    log.write_text("".join(f"{now - i:.3f} svc.example.com 200 {(i + 1) / 10:.1f}\n" for i in range(10)))
    sc = StatsCollector(str(log))
    st = sc.collect()["svc.example.com"]
    assert st[30]["requests"] == 10
    assert abs(st[30]["request_time"] - 0.55) < 1e-6
    # rotation: a new, shorter file is read from the start
    log.write_text(f"{time.time():.3f} svc.example.com 200 1.0\n")
    assert sc.collect()["svc.example.com"][30]["requests"] == 11


def test_model_proxy_openai_and_tgi(gw, upstream):
    ctl = TestClient(make_app(gw))
    _register(ctl, upstream, run="llm", model={"name": "llama", "format": "openai", "prefix": "/v1"})
    _register(ctl, upstream, run="tgi", model={"name": "llama-tgi", "format": "tgi"})
    names = {m["id"] for m in ctl.get("/api/models/main/models").json()["data"]}
    assert names == {"llama", "llama-tgi"}
    r = ctl.post("/api/models/main/chat/completions",
                 json={"model": "llama", "messages": [{"role": "user", "content": "ping"}]})
    assert r.json()["choices"][0]["message"]["content"] == "pong"
    r = ctl.post("/api/models/main/chat/completions",
                 json={"model": "llama-tgi", "messages": [{"role": "user", "content": "hi"}], "max_tokens": 8})
    assert r.json()["choices"][0]["message"]["content"] == "tgi-answer"
    assert ctl.post("/api/models/main/chat/completions", json={"model": "nope", "messages": []}).status_code == 404


def test_nginx_render_and_rollback(tmp_path):
    ng = Nginx(conf_dir=str(tmp_path / "sites"), access_log=str(tmp_path / "a.log"), reload_cmd=["true"],
               test_cmd=["true"])
    reg = Registry()
    svc = reg.register_service("main", "svc", "svc.example.com", auth=True)
    reg.add_replica("main", "svc", Replica(id="1", app_port=8000, internal_ip="10.1.2.3"))
    reg.add_replica("main", "svc", Replica(id="2", app_port=8000, mode="ssh", socket="/tmp/r2.sock",
                                           ssh_host="u@h"))
    ng.apply_service(svc)
    text = (tmp_path / "sites" / "80-svc.example.com.conf").read_text()
    assert "server 10.1.2.3:8000;" in text and "server unix:/tmp/r2.sock;" in text
    assert "auth_request /_dstack_auth;" in text and "server_name svc.example.com;" in text
    # a failing `nginx -t` restores the previous file
    ng.test_cmd = ["false"]
    reg.remove_replica("main", "svc", "1")
    with pytest.raises(Exception):
        ng.apply_service(svc)
    assert (tmp_path / "sites" / "80-svc.example.com.conf").read_text() == text
