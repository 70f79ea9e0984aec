"""Gateway application (reference: ``P/gateway/app.py:53-89``, routers ``P/gateway/routers/
{auth,config,registry,stats}.py``, ``P/gateway/auth.py``, ``P/gateway/services/server_client.py``).

Two ASGI apps:

* the **control app** (``make_app``, loopback :8000, reached by the server over SSH): registry
  API, stats, config, token auth for nginx ``auth_request``, and the OpenAI-compatible model API
  of each project's entrypoint;
* the **data plane** (``make_dataplane_app``): a Host-routed streaming reverse proxy used when
  nginx is not installed (dev / CI / small on-prem setups).  With nginx it is not started.
"""

from __future__ import annotations

import asyncio
import itertools
import logging
import os
import subprocess
import time
from pathlib import Path
from typing import Dict, Optional

import httpx
from fastapi import APIRouter, FastAPI, Request
from fastapi.responses import JSONResponse, Response, StreamingResponse
from pydantic import BaseModel
from starlette.background import BackgroundTask

from dstack_amd.proxy.gateway.nginx import Nginx
from dstack_amd.proxy.gateway.registry import Registry, RegistryError, Replica
from dstack_amd.proxy.gateway.stats import WINDOWS, StatsCollector
from dstack_amd.proxy.lib.model_proxy import make_client, models_response

logger = logging.getLogger(__name__)


# ---- request bodies ---------------------------------------------------------------------------
class RegisterServiceBody(BaseModel):
    run_name: str
    domain: str
    https: bool = False
    auth: bool = True
    client_max_body_size: int = 64 * 2**20
    options: dict = {}


class RegisterReplicaBody(BaseModel):
    job_id: str
    app_port: int
    ssh_host: Optional[str] = None
    ssh_port: int = 22
    ssh_proxy: Optional[str] = None
    internal_ip: Optional[str] = None
    direct: bool = True


class RegisterEntrypointBody(BaseModel):
    domain: str
    https: bool = False


class ConfigBody(BaseModel):
    server_url: Optional[str] = None
    acme_server: Optional[str] = None
    acme_eab_kid: Optional[str] = None
    acme_eab_hmac_key: Optional[str] = None


# ---- auth (reference: GatewayProxyAuthProvider, 60 s cache) ----------------------------------
class TokenAuth:
    TTL = 60.0

    def __init__(self, server_url: Optional[str] = None):
        self.server_url = server_url
        self._cache: Dict[tuple, float] = {}

    async def is_member(self, project: str, token: Optional[str]) -> bool:
        if not token:
            return False
        key = (project, token)
        t = self._cache.get(key)
        if t is not None and time.time() - t < self.TTL:
            return True
        if not self.server_url:
            return False
        try:
            async with httpx.AsyncClient(timeout=10) as c:
                r = await c.post(f"{self.server_url}/api/projects/{project}/get",
                                 headers={"Authorization": f"Bearer {token}"})
        except httpx.HTTPError:
            return False
        if r.status_code == 200:
            self._cache[key] = time.time()
            return True
        return False


def _bearer(request: Request) -> Optional[str]:
    a = request.headers.get("authorization", "")
    return a[7:].strip() if a.lower().startswith("bearer ") else None


# ---- replica connections ---------------------------------------------------------------------
class ReplicaConnections:
    """``ssh -N -L <sock>:localhost:<port>`` per non-direct replica (reference: ServiceConnection)."""

    def __init__(self, sock_dir: Path, identity_file: Optional[str] = None, connect_timeout: float = 20.0):
        self.sock_dir = sock_dir
        self.identity_file = identity_file
        self.connect_timeout = connect_timeout
        self._procs: Dict[str, subprocess.Popen] = {}

    def open(self, rep: Replica) -> Replica:
        if rep.mode != "ssh" or not rep.ssh_host:
            return rep
        self.sock_dir.mkdir(parents=True, exist_ok=True)
        rep.socket = str(self.sock_dir / f"replica-{rep.id}.sock")
        if os.path.exists(rep.socket):
            os.unlink(rep.socket)
        host, _, user_host = rep.ssh_host.rpartition("@")
        cmd = ["ssh", "-N", "-o", "StrictHostKeyChecking=no", "-o", "UserKnownHostsFile=/dev/null",
               "-o", "ExitOnForwardFailure=yes", "-o", "ServerAliveInterval=15", "-p", str(rep.ssh_port),
               "-L", f"{rep.socket}:localhost:{rep.app_port}"]
        if self.identity_file:
            cmd += ["-i", self.identity_file]
        if rep.ssh_proxy:
            cmd += ["-J", rep.ssh_proxy]
        cmd.append(rep.ssh_host)
        proc = subprocess.Popen(cmd, stdin=subprocess.DEVNULL, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
        _ = host, user_host
        # the forward is up when its socket exists; an ssh that exits first (bad key, host down) is a
        # registration error, not a replica that nginx would route to a dead socket
        deadline = time.time() + self.connect_timeout
        while not os.path.exists(rep.socket):
            if proc.poll() is not None:
                err = proc.stderr.read().decode(errors="ignore").strip() if proc.stderr else ""
                raise RegistryError(f"cannot connect to replica {rep.id} ({rep.ssh_host}): {err[-300:] or 'ssh exited'}")
            if time.time() > deadline:
                proc.kill()
                raise RegistryError(f"cannot connect to replica {rep.id} ({rep.ssh_host}): timed out")
            time.sleep(0.05)
        self._procs[rep.id] = proc
        return rep

    def close(self, rep_id: str):
        p = self._procs.pop(rep_id, None)
        if p is not None:
            p.terminate()
            try:
                p.wait(5)
            except subprocess.TimeoutExpired:
                p.kill()

    def close_all(self):
        for rid in list(self._procs):
            self.close(rid)


class Gateway:
    def __init__(self, state_dir: Path, nginx: Optional[Nginx] = None, server_url: Optional[str] = None,
                 identity_file: Optional[str] = None):
        self.state_dir = state_dir
        self.registry = Registry(state_dir / "state-v2.json")
        self.nginx = nginx
        self.stats = StatsCollector(nginx.access_log if nginx else None)
        self.auth = TokenAuth(server_url or self.registry.acme.get("server_url"))
        self.conns = ReplicaConnections(state_dir / "sockets", identity_file)
        self._rr: Dict[str, itertools.count] = {}
        self.http = httpx.AsyncClient(timeout=httpx.Timeout(300, connect=10))
        # restore: re-open tunnels and re-render sites from the persisted state
        for svc in self.registry.services.values():
            for rep in svc.replicas.values():
                try:
                    self.conns.open(rep)
                except RegistryError as e:  # the server re-registers what it still runs
                    logger.warning("replica %s not reconnected: %s", rep.id, e)
            self._apply_site(svc)
        if nginx is not None:
            for ep in self.registry.entrypoints.values():
                nginx.apply_entrypoint(ep)

    def _apply_site(self, svc):
        if self.nginx is not None:
            self.nginx.apply_service(svc)

    def pick_replica(self, svc) -> Optional[Replica]:
        reps = list(svc.replicas.values())
        if not reps:
            return None
        n = next(self._rr.setdefault(svc.key, itertools.count()))
        return reps[n % len(reps)]

    def replica_client(self, rep: Replica):
        if rep.mode == "ssh" and rep.socket:
            return httpx.AsyncClient(transport=httpx.AsyncHTTPTransport(uds=rep.socket), timeout=300), "http://replica"
        return self.http, f"http://{rep.upstream()}"


def make_app(gw: Gateway) -> FastAPI:
    from contextlib import asynccontextmanager

    @asynccontextmanager
    async def lifespan(_app):
        # state was restored when the Gateway was built (sites re-rendered, replica tunnels reopened);
        # on shutdown the tunnels and the upstream client go away with the process
        yield
        gw.conns.close_all()
        await gw.http.aclose()

    app = FastAPI(title="dstack-amd gateway", docs_url=None, redoc_url=None, lifespan=lifespan)
    r = APIRouter()

    @r.get("/api/healthcheck")
    async def healthcheck():
        from dstack_amd import __version__

        # ``version`` is what update.sh and the server's init_gateways compare against
        return {"service": "dstack-gateway", "version": __version__, "services": len(gw.registry.services)}

    @r.post("/api/config")
    async def config(body: ConfigBody):
        if body.server_url:
            gw.auth.server_url = body.server_url
        gw.registry.acme.update({k: v for k, v in body.model_dump().items() if v is not None})
        gw.registry.save()
        return {}

    @r.post("/api/registry/{project}/services/register")
    async def register_service(project: str, body: RegisterServiceBody):
        model = (body.options.get("openai") or {}).get("model")
        try:
            svc = gw.registry.register_service(project, body.run_name, body.domain, body.https, body.auth,
                                               body.client_max_body_size, model)
            await asyncio.to_thread(gw._apply_site, svc)
        except RegistryError as e:
            return JSONResponse({"detail": str(e)}, status_code=400)
        return {}

    @r.post("/api/registry/{project}/services/{run_name}/unregister")
    async def unregister_service(project: str, run_name: str):
        try:
            svc = gw.registry.unregister_service(project, run_name)
        except RegistryError as e:
            return JSONResponse({"detail": str(e)}, status_code=400)
        for rid in svc.replicas:
            gw.conns.close(rid)
        if gw.nginx is not None:
            await asyncio.to_thread(gw.nginx.remove, svc.domain)
        return {}

    @r.post("/api/registry/{project}/services/{run_name}/replicas/register")
    async def register_replica(project: str, run_name: str, body: RegisterReplicaBody):
        rep = Replica(id=body.job_id, app_port=body.app_port, ssh_host=body.ssh_host, ssh_port=body.ssh_port,
                      ssh_proxy=body.ssh_proxy, internal_ip=body.internal_ip,
                      mode="direct" if body.direct or not body.ssh_host else "ssh")
        svc = gw.registry.get_service(project, run_name)
        if svc is None:
            return JSONResponse({"detail": f"service {project}/{run_name} is not registered"}, status_code=400)
        if rep.id in svc.replicas:
            return JSONResponse({"detail": f"replica {rep.id} of {project}/{run_name} is already registered"},
                                status_code=400)
        try:
            await asyncio.to_thread(gw.conns.open, rep)
            svc = gw.registry.add_replica(project, run_name, rep)
            await asyncio.to_thread(gw._apply_site, svc)
        except RegistryError as e:
            gw.conns.close(rep.id)
            return JSONResponse({"detail": str(e)}, status_code=400)
        return {}

    @r.post("/api/registry/{project}/services/{run_name}/replicas/{job_id}/unregister")
    async def unregister_replica(project: str, run_name: str, job_id: str):
        try:
            gw.registry.remove_replica(project, run_name, job_id)
        except RegistryError as e:
            return JSONResponse({"detail": str(e)}, status_code=400)
        gw.conns.close(job_id)
        svc = gw.registry.get_service(project, run_name)
        if svc is not None:
            await asyncio.to_thread(gw._apply_site, svc)
        return {}

    @r.post("/api/registry/{project}/entrypoints/register")
    async def register_entrypoint(project: str, body: RegisterEntrypointBody):
        ep = gw.registry.register_entrypoint(project, body.domain, body.https)
        if gw.nginx is not None:
            await asyncio.to_thread(gw.nginx.apply_entrypoint, ep)
        return {}

    @r.get("/api/stats/collect")
    async def collect_stats():
        per_host = gw.stats.collect()
        out = []
        for svc in gw.registry.services.values():
            st = per_host.get(svc.domain.lower(), {w: {"requests": 0, "request_time": 0.0} for w in WINDOWS})
            out.append({"project_name": svc.project, "run_name": svc.run_name,
                        "stats": {str(w): v for w, v in st.items()}})
        return out

    @r.get("/api/auth/{project}")
    async def auth(project: str, request: Request):
        if await gw.auth.is_member(project, _bearer(request)):
            return Response(status_code=200)
        return Response(status_code=403)

    @r.get("/api/models/{project}/models")
    async def list_models(project: str):
        return models_response([{**s.model, "created": 0} for s in gw.registry.project_models(project)])

    @r.post("/api/models/{project}/chat/completions")
    async def chat(project: str, request: Request):
        body = await request.json()
        svc = next((s for s in gw.registry.project_models(project) if s.model.get("name") == body.get("model")), None)
        if svc is None:
            return JSONResponse({"detail": f"model {body.get('model')} not found"}, status_code=404)
        if svc.auth and not await gw.auth.is_member(project, _bearer(request)):
            return JSONResponse({"detail": "unauthorized"}, status_code=403)
        rep = gw.pick_replica(svc)
        if rep is None:
            return JSONResponse({"detail": "no replicas"}, status_code=503)
        _, base = gw.replica_client(rep)
        client = make_client(svc.model, base if rep.mode == "direct" else f"http://{rep.upstream()}")
        start = time.time()
        if body.get("stream"):
            gw.stats.record(svc.domain, 0.0)
            return StreamingResponse(client.stream(body), media_type="text/event-stream")
        out = await client.generate(body)
        gw.stats.record(svc.domain, time.time() - start)
        return out

    app.include_router(r)
    return app


def make_dataplane_app(gw: Gateway) -> FastAPI:
    """Host-routed streaming reverse proxy (the nginx site semantics, in-process)."""
    app = FastAPI(docs_url=None, redoc_url=None, openapi_url=None)

    @app.api_route("/{path:path}", methods=["GET", "POST", "PUT", "PATCH", "DELETE", "OPTIONS", "HEAD"])
    async def proxy(path: str, request: Request):
        host = request.headers.get("host", "")
        svc = gw.registry.service_by_domain(host)
        if svc is None:
            ep = gw.registry.entrypoint_by_domain(host)
            if ep is not None:
                return await _forward(request, gw.http, f"http://127.0.0.1:{request.app.state.control_port}",
                                      f"/api/models/{ep.project}/{path}", host, None)
            return JSONResponse({"detail": f"unknown host {host}"}, status_code=404)
        if svc.auth and not await gw.auth.is_member(svc.project, _bearer(request)):
            return JSONResponse({"detail": "unauthorized"}, status_code=403)
        rep = gw.pick_replica(svc)
        if rep is None:
            return JSONResponse({"detail": "no replicas"}, status_code=503)
        client, base = gw.replica_client(rep)
        return await _forward(request, client, base, "/" + path, host, gw.stats)

    app.state.control_port = 8000
    return app


async def _forward(request: Request, client: httpx.AsyncClient, base: str, path: str, host: str,
                   stats: Optional[StatsCollector]):
    url = base + path + (("?" + request.url.query) if request.url.query else "")
    headers = {k: v for k, v in request.headers.items() if k.lower() not in ("content-length",)}
    start = time.time()
    try:
        upstream = await client.send(client.build_request(request.method, url, headers=headers,
                                                          content=await request.body()), stream=True)
    except httpx.HTTPError as e:
        return JSONResponse({"detail": f"upstream error: {e}"}, status_code=502)
    if stats is not None:
        stats.record(host, time.time() - start)
    hdrs = {k: v for k, v in upstream.headers.items()
            if k.lower() not in ("content-length", "transfer-encoding", "connection", "content-encoding")}
    return StreamingResponse(upstream.aiter_raw(), status_code=upstream.status_code, headers=hdrs,
                             background=BackgroundTask(upstream.aclose))
