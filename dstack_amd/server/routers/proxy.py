"""In-server service proxy and OpenAI model proxy (reference: ``S/services/proxy/services/
service_proxy.py:21-135``, ``S/services/proxy/repo.py``; routes ``/proxy/services/{p}/{run}/...``
and ``/proxy/models/{p}/...`` — ``S/app.py:184-185``).

Replicas are resolved from the DB per request (running jobs of the run), load-balanced
round-robin; remote replicas are reached through the pooled SSH port forwards.  Request counts
and latencies feed the RPS autoscaler.
"""

from __future__ import annotations

import asyncio
import itertools
import json
import time
from http.cookiejar import CookieJar
from typing import Dict, List, Optional, Tuple

import httpx
from fastapi import APIRouter, Request
from fastapi.responses import JSONResponse, RedirectResponse, Response, StreamingResponse
from starlette.concurrency import run_in_threadpool
from starlette.background import BackgroundTask

from dstack_amd.core.models.configurations import ServiceConfiguration
from dstack_amd.core.models.runs import JobStatus, RunSpec, RunStatus
from dstack_amd.proxy.lib.model_proxy import make_client, models_response
from dstack_amd.server.db import session_scope
from dstack_amd.server.models import RunModel
from dstack_amd.server.services import jobs as jobs_services
from dstack_amd.server.services.projects import get_member_role, get_project_by_name
from dstack_amd.server.services.services import get_request_stats
from dstack_amd.server.services.users import get_user_by_token

router = APIRouter(tags=["proxy"])
_rr: Dict[str, itertools.count] = {}


class _NoCookies(CookieJar):
    """The upstream client is shared by every downstream user: it must never remember a
    ``Set-Cookie`` (that would hand one user's session to the next); cookies travel only in the
    request/response headers."""

    def extract_cookies(self, response, request):
        pass

    def set_cookie(self, cookie):
        pass


_clients: Dict[int, httpx.AsyncClient] = {}


def _upstream_client() -> httpx.AsyncClient:
    """One pooled client per event loop (connections are bound to the loop that opened them)."""
    from dstack_amd.server import settings

    loop = asyncio.get_running_loop()
    c = _clients.get(id(loop))
    if c is None or c.is_closed:
        c = httpx.AsyncClient(timeout=httpx.Timeout(settings.PROXY_UPSTREAM_TIMEOUT, connect=10),
                              cookies=httpx.Cookies(_NoCookies()), follow_redirects=False)
        _clients[id(loop)] = c
    return c


# hop-by-hop headers (RFC 9110 7.6.1) are never forwarded; the body length is re-derived
_HOP = {"connection", "keep-alive", "proxy-authenticate", "proxy-authorization", "te", "trailer",
        "transfer-encoding", "upgrade"}


def _replica_urls(s, run: RunModel, conf: ServiceConfiguration) -> List[str]:
    from dstack_amd.server.services.runner.client import port_base_url

    urls = []
    for j in run.jobs:
        if j.status != JobStatus.RUNNING.value:
            continue
        jpd = jobs_services.job_jpd(j)
        if jpd is None:
            continue
        port = conf.port.container_port
        jrd = jobs_services.job_jrd(j)
        if jrd and jrd.ports:
            port = int(jrd.ports.get(port, jrd.ports.get(str(port), port)))
        urls.append(port_base_url(jpd, run.project.ssh_private_key, port))
    return urls


def _resolve(project_name: str, run_name: str, token: Optional[str]) -> Tuple[Optional[str], Optional[dict], int, str]:
    """-> (replica_url, model_dict, status, error)"""
    with session_scope() as s:
        project = get_project_by_name(s, project_name)
        not_found = f"Service {project_name}/{run_name} not found"
        if project is None:
            return None, None, 404, not_found
        run = s.query(RunModel).filter(RunModel.project_id == project.id, RunModel.run_name == run_name,
                                       RunModel.deleted == False).order_by(RunModel.submitted_at.desc()).first()  # noqa
        if run is None or RunStatus(run.status).is_finished():
            return None, None, 404, not_found
        spec = RunSpec.model_validate_json(run.run_spec)
        conf = spec.configuration
        if not isinstance(conf, ServiceConfiguration):
            return None, None, 404, not_found
        if conf.auth:
            user = get_user_by_token(s, token) if token else None
            if user is None or (user.global_role != "admin" and get_member_role(project, user) is None):
                return None, None, 403, "Access denied"
        urls = _replica_urls(s, run, conf)
        if not urls:
            return None, None, 503, f"Service {project_name}/{run_name} has no running replicas"
        key = str(run.id)
        n = next(_rr.setdefault(key, itertools.count()))
        model = conf.model.model_dump() if conf.model else None
        meta = {"run_id": key, "strip_prefix": conf.strip_prefix}
        return urls[n % len(urls)], (model | meta if model else meta), 200, ""


def _token(request: Request) -> Optional[str]:
    a = request.headers.get("authorization", "")
    return a[7:].strip() if a.lower().startswith("bearer ") else None


@router.api_route("/proxy/services/{project_name}/{run_name}", methods=["GET", "HEAD"], include_in_schema=False)
async def service_root_redirect(project_name: str, run_name: str, request: Request):
    """``.../run`` -> ``.../run/`` (308 keeps the method), so relative links resolve under the prefix."""
    url = request.url.replace(path=request.url.path + "/")
    return RedirectResponse(str(url), status_code=308)


@router.api_route("/proxy/services/{project_name}/{run_name}/{path:path}",
                  methods=["GET", "POST", "PUT", "PATCH", "DELETE", "OPTIONS", "HEAD"], include_in_schema=False)
async def service_proxy(project_name: str, run_name: str, path: str, request: Request):
    """Forward one request to a replica: original ``Host`` and headers minus hop-by-hop ones, body
    streamed both ways, status and headers passed through (``Content-Length``/``-Encoding``
    included -- the body is relayed undecoded), no cookie state kept between users, 504 when the
    replica does not answer in ``DSTACK_PROXY_UPSTREAM_TIMEOUT``."""
    url, meta, status, err = await run_in_threadpool(_resolve, project_name, run_name, _token(request))
    if url is None:
        return JSONResponse({"detail": err}, status_code=status)
    prefix = f"/proxy/services/{project_name}/{run_name}"
    target = f"{url}/{path}" if meta["strip_prefix"] else f"{url}{prefix}/{path}"
    if request.url.query:
        target += "?" + request.url.query
    # a sized body keeps its Content-Length (streamed, not re-chunked: not every replica server
    # reads chunked uploads); an unsized one goes chunked
    headers = [(k, v) for k, v in request.headers.items() if k.lower() not in _HOP]
    client = _upstream_client()
    start = time.time()
    body = request.stream() if request.method not in ("GET", "HEAD", "OPTIONS") else None
    req = client.build_request(request.method, target, headers=headers, content=body)
    try:
        upstream = await client.send(req, stream=True)
    except httpx.TimeoutException:
        return JSONResponse({"detail": "Timed out requesting upstream"}, status_code=504)
    except httpx.HTTPError as e:
        return JSONResponse({"detail": f"Error requesting upstream: {e}"}, status_code=502)
    get_request_stats().record(meta["run_id"], time.time() - start)
    resp_headers = [(k, v) for k, v in upstream.headers.multi_items() if k.lower() not in _HOP]
    if request.method == "HEAD" or upstream.status_code in (204, 304):
        await upstream.aclose()
        r = Response(status_code=upstream.status_code)
        r.raw_headers = [(k.lower().encode("latin-1"), v.encode("latin-1")) for k, v in resp_headers]
        return r
    r = StreamingResponse(upstream.aiter_raw(), status_code=upstream.status_code,
                          background=BackgroundTask(upstream.aclose))
    r.raw_headers = [(k.lower().encode("latin-1"), v.encode("latin-1")) for k, v in resp_headers]
    return r


def _project_models(project_name: str) -> List[dict]:
    out = []
    with session_scope() as s:
        project = get_project_by_name(s, project_name)
        if project is None:
            return out
        for run in s.query(RunModel).filter(RunModel.project_id == project.id, RunModel.deleted == False):  # noqa
            if RunStatus(run.status).is_finished():
                continue
            conf = RunSpec.model_validate_json(run.run_spec).configuration
            if isinstance(conf, ServiceConfiguration) and conf.model is not None:
                out.append({**conf.model.model_dump(), "run_name": run.run_name,
                            "created": run.submitted_at.timestamp()})
    return out


@router.get("/proxy/models/{project_name}/models")
async def list_models(project_name: str):
    models = await run_in_threadpool(_project_models, project_name)
    return models_response(models)


@router.post("/proxy/models/{project_name}/chat/completions")
async def chat_completions(project_name: str, request: Request):
    body = await request.json()
    models = await run_in_threadpool(_project_models, project_name)
    model = next((m for m in models if m["name"] == body.get("model")), None)
    if model is None:
        return JSONResponse({"detail": f"model {body.get('model')} not found"}, status_code=404)
    url, meta, status, err = await run_in_threadpool(_resolve, project_name, model["run_name"], _token(request))
    if url is None:
        return JSONResponse({"detail": err}, status_code=status)
    client = make_client(model, url)
    start = time.time()
    if body.get("stream"):
        get_request_stats().record(meta["run_id"], 0.0, start)
        return StreamingResponse(client.stream(body), media_type="text/event-stream")
    out = await client.generate(body)
    get_request_stats().record(meta["run_id"], time.time() - start)
    return Response(json.dumps(out), media_type="application/json")
