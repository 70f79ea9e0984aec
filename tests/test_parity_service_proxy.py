"""The in-server service proxy (``/proxy/services/{project}/{run}/...``), case by case against the
reference's ``server/services/proxy/routers/test_service_proxy.py`` (mapping:
``docs/reference/test-parity.md``). The replica is a small httpbin-like HTTP server on 127.0.0.1
(the reference mocks its replica client with pytest-httpbin, which this image does not have)."""

from __future__ import annotations

import json
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Optional
from urllib.parse import parse_qsl, urlsplit

import pytest

from tests.conftest import ADMIN_TOKEN


class _Bin(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"

    def log_message(self, *a):
        pass

    def version_string(self):
        return "Test-HTTPBIN/1.0"

    def _send(self, code, body: bytes = b"", headers=()):
        self.send_response(code)
        for k, v in headers:
            self.send_header(k, v)
        if code not in (204, 304):
            self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        if body and self.command != "HEAD" and code not in (204, 304):
            self.wfile.write(body)

    def _json(self, obj, headers=()):
        self._send(200, json.dumps(obj).encode(), [("Content-Type", "application/json"), *headers])

    def _handle(self):
        u = urlsplit(self.path)
        n = int(self.headers.get("Content-Length") or 0)
        data = self.rfile.read(n).decode() if n else ""
        if self.server.report_path:  # strip_prefix cases: answer with the path the replica saw
            self._send(200, self.path.encode(), [("Content-Type", "text/plain")])
            return
        if self.command == "OPTIONS":
            self._send(200, b"", [("Allow", "HEAD, GET, OPTIONS")])
            return
        if u.path.startswith("/status/"):
            self._send(int(u.path.rsplit("/", 1)[1]))
            return
        if u.path.startswith("/delay/"):
            time.sleep(float(u.path.rsplit("/", 1)[1]))
            self._json({})
            return
        if u.path == "/cookies/set":
            self._send(200, b"{}", [("Set-Cookie", f"{k}={v}; Path=/") for k, v in parse_qsl(u.query)])
            return
        if u.path == "/cookies":
            jar = dict(c.strip().split("=", 1) for c in (self.headers.get("Cookie") or "").split(";") if "=" in c)
            self._json({"cookies": jar})
            return
        self._json({"url": f"http://{self.headers['Host']}{self.path}",
                    "args": dict(parse_qsl(u.query, keep_blank_values=True)),
                    "headers": {k.title() if k.lower() != "user-agent" else "User-Agent": v
                                for k, v in self.headers.items()},
                    "data": data})

    do_GET = do_POST = do_PUT = do_PATCH = do_DELETE = do_HEAD = do_OPTIONS = _handle


@pytest.fixture
def upstream():
    srv = ThreadingHTTPServer(("127.0.0.1", 0), _Bin)
    srv.daemon_threads = True
    srv.report_path = False
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    yield srv
    srv.shutdown()
    srv.server_close()


@pytest.fixture
def app(db, upstream, monkeypatch):
    from dstack_amd.server import settings
    from dstack_amd.server.app import create_app
    from dstack_amd.server.routers import proxy

    monkeypatch.setattr(settings, "PROXY_UPSTREAM_TIMEOUT", 1.0)
    monkeypatch.setattr(proxy, "_replica_urls",
                        lambda s, run, conf: [f"http://127.0.0.1:{upstream.server_address[1]}"])
    return create_app(start_background=False)


def _tc(app, token: Optional[str] = ADMIN_TOKEN):
    from fastapi.testclient import TestClient

    c = TestClient(app, base_url="http://test-host:8888")
    if token is not None:
        c.headers.update({"Authorization": f"Bearer {token}"})
    return c


def _service(c, name="httpbin", **kw):
    r = c.post("/api/project/main/repos/init", json={"repo_id": "virt", "repo_info": {"repo_type": "virtual"}})
    assert r.status_code == 200, r.text
    conf = {"type": "service", "commands": ["serve"], "port": 80, **kw}
    r = c.post("/api/project/main/runs/submit", json={"run_spec": {
        "run_name": name, "repo_id": "virt", "repo_data": {"repo_type": "virtual"}, "configuration": conf,
        "ssh_key_pub": ""}})
    assert r.status_code == 200, r.text


@pytest.mark.parametrize("method", ["get", "post", "put", "patch", "delete"])
def test_proxy_forwards_method_url_headers_body(app, method):
    with _tc(app) as c:
        _service(c, auth=False)
        body = "." * (4 << 20) if method not in ("get", "delete") else None  # 4 MiB streamed through
        r = c.request(method.upper(), f"/proxy/services/main/httpbin/{method}?a=b&c=",
                      headers={"User-Agent": "test-ua"}, content=body)
        assert r.status_code == 200, r.text
        assert r.headers["server"].startswith("Test-HTTPBIN")
        out = r.json()
        assert out["url"] == f"http://test-host:8888/{method}?a=b&c="  # original Host, prefix stripped
        assert out["args"] == {"a": "b", "c": ""}
        assert out["headers"]["Host"] == "test-host:8888"
        assert out["headers"]["User-Agent"] == "test-ua"
        if body is not None:
            assert out["data"] == body


def test_proxy_method_head(app):
    with _tc(app) as c:
        _service(c, auth=False)
        g = c.get("/proxy/services/main/httpbin/")
        h = c.head("/proxy/services/main/httpbin/")
        assert g.status_code == h.status_code == 200
        assert h.headers["content-length"] == g.headers["content-length"] and int(h.headers["content-length"]) > 0
        assert h.content == b""


def test_proxy_method_options(app):
    with _tc(app) as c:
        _service(c, auth=False)
        r = c.options("/proxy/services/main/httpbin/get")
        assert r.status_code == 200
        assert set(r.headers["allow"].split(", ")) == {"HEAD", "GET", "OPTIONS"}
        assert r.content == b""


@pytest.mark.parametrize("code", [204, 304, 418, 503])
def test_proxy_status_codes(app, code):
    with _tc(app) as c:
        _service(c, auth=False)
        assert c.get(f"/proxy/services/main/httpbin/status/{code}").status_code == code


def test_proxy_does_not_leak_cookies_between_clients(app):
    with _tc(app) as c1, _tc(app) as c2:
        _service(c1, auth=False)
        url = "/proxy/services/main/httpbin/cookies"
        c1.get(url + "/set?a=1")
        c1.get(url + "/set?b=2")
        c2.get(url + "/set?a=3")
        assert c1.get(url).json()["cookies"] == {"a": "1", "b": "2"}
        assert c2.get(url).json()["cookies"] == {"a": "3"}


def test_proxy_gateway_timeout(app):
    with _tc(app) as c:
        _service(c, auth=False)
        r = c.get("/proxy/services/main/httpbin/delay/3")  # upstream timeout is 1 s here
        assert r.status_code == 504
        assert r.json()["detail"] == "Timed out requesting upstream"


def test_proxy_run_not_found(app):
    with _tc(app) as c:
        _service(c, name="test-run", auth=False)
        r = c.get("/proxy/services/main/unknown/")
        assert r.status_code == 404 and r.json()["detail"] == "Service main/unknown not found"


def test_proxy_project_not_found(app):
    with _tc(app) as c:
        r = c.get("/proxy/services/unknown/test-run/")
        assert r.status_code == 404 and r.json()["detail"] == "Service unknown/test-run not found"


def test_redirect_to_service_root(app):
    with _tc(app) as c:
        _service(c, auth=False)
        url = "http://test-host:8888/proxy/services/main/httpbin"
        r = c.get(url, follow_redirects=False)
        assert r.status_code == 308 and r.headers["location"] == url + "/"
        r = c.get(url, follow_redirects=True)
        assert r.status_code == 200 and str(r.url) == url + "/"


@pytest.mark.parametrize("token,status", [("correct", 200), ("incorrect-token", 403), ("", 403), (None, 403)])
def test_auth(app, token, status):
    with _tc(app) as admin:
        _service(admin, auth=True)
    tok = ADMIN_TOKEN if token == "correct" else token
    with _tc(app, token=None) as c:
        headers = {"Authorization": f"Bearer {tok}"} if tok is not None else {}
        assert c.get("/proxy/services/main/httpbin/", headers=headers).status_code == status


@pytest.mark.parametrize("strip,downstream,upstream_path", [
    (True, "/proxy/services/main/my-run/", "/"),
    (True, "/proxy/services/main/my-run/a/b", "/a/b"),
    (False, "/proxy/services/main/my-run/", "/proxy/services/main/my-run/"),
    (False, "/proxy/services/main/my-run/a/b", "/proxy/services/main/my-run/a/b"),
])
def test_strip_prefix(app, upstream, strip, downstream, upstream_path):
    upstream.report_path = True
    with _tc(app) as c:
        _service(c, name="my-run", auth=False, strip_prefix=strip)
        r = c.get(downstream)
        assert r.status_code == 200 and r.text == upstream_path
