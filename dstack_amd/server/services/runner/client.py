"""HTTP clients for the native agents (reference: ``S/services/runner/client.py:47-389``) and the
connection logic that reaches them: loopback for the ``local`` backend, pooled SSH port forwards
for remote hosts (``core/services/ssh/tunnel.py``)."""

from __future__ import annotations

import json
import re
from typing import Any, Dict, List, Optional, Tuple

import httpx

from dstack_amd.core.backends.base import DSTACK_RUNNER_HTTP_PORT, DSTACK_SHIM_HTTP_PORT
from dstack_amd.core.errors import RunnerError, SSHError
from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.runs import ClusterInfo, JobProvisioningData, JobRuntimeData, JobSpec, RunSpec
from dstack_amd.core.services.ssh.tunnel import SSHTarget, get_tunnel_pool

REQUEST_TIMEOUT = 15.0

_clients: Dict[str, httpx.Client] = {}


def _client(base_url: str, transport: Optional[httpx.BaseTransport] = None) -> httpx.Client:
    if transport is not None:  # tests: an in-process transport, never pooled
        return httpx.Client(base_url=base_url, timeout=REQUEST_TIMEOUT, transport=transport)
    c = _clients.get(base_url)
    if c is None:
        c = httpx.Client(base_url=base_url, timeout=REQUEST_TIMEOUT)
        _clients[base_url] = c
    return c


# shim HTTP API generations: 1 = tasks API without the GPU health probe endpoints,
# 2 = + ``/api/gpu_health`` (probe state, off-path re-probe) and preemption ("interrupted")
SHIM_LATEST_API_VERSION = 2
# final shim releases older than this speak API 1 (a shim that reports ``api_version`` wins)
SHIM_API_V2_MIN_VERSION = (0, 1, 0)

_FINAL_VERSION = re.compile(r"^(\d+)\.(\d+)(?:\.(\d+))?(?:\.\d+)*(?:\+[0-9A-Za-z.]+)?$")


def parse_version(value: str) -> Optional[Tuple[int, int, int]]:
    """``major.minor[.patch[.more]][+local]`` -> ``(major, minor, patch)``; None for anything that
    is not a final release (pre/dev/rc, major-only build numbers, ``latest``, garbage) -- such
    agents are local or CI builds and are assumed to speak the latest API
    (reference: ``S/services/runner/client.py`` ``_parse_version``)."""
    m = _FINAL_VERSION.match(value or "")
    if m is None:
        return None
    return int(m.group(1)), int(m.group(2)), int(m.group(3) or 0)


class ShimHTTPError(RunnerError):
    """A non-2xx answer from the shim, with the HTTP status kept for callers that branch on it."""

    def __init__(self, status_code: int, message: str):
        super().__init__(message)
        self.status_code = status_code
        self.message = message

    def __repr__(self) -> str:
        return f"ShimHTTPError({self.status_code})"


class ShimClient:
    def __init__(self, base_url: str, transport: Optional[httpx.BaseTransport] = None):
        self.base_url = base_url
        self.c = _client(base_url, transport)

    # -- API negotiation ------------------------------------------------------------------
    def _negotiate(self) -> None:
        """One healthcheck call fixes the agent's version and API generation for this client."""
        data = self.healthcheck() or {}
        self._shim_version = parse_version(str(data.get("version", "")))
        api = data.get("api_version")
        if isinstance(api, int):
            self._api_version = api
        elif self._shim_version is not None and self._shim_version < SHIM_API_V2_MIN_VERSION:
            self._api_version = 1
        else:
            self._api_version = SHIM_LATEST_API_VERSION

    @property
    def api_version(self) -> int:
        if not hasattr(self, "_api_version"):
            self._negotiate()
        return self._api_version

    def _request(self, method: str, path: str, **kw) -> httpx.Response:
        return self.c.request(method, path, **kw)

    @staticmethod
    def _raise_for_status(r: httpx.Response) -> None:
        if r.is_success:
            return
        kind = "Client" if r.status_code < 500 else "Server"
        msg = f"{r.status_code} {kind} Error: {r.reason_phrase} for url: {r.url}"
        body = r.text.strip()
        if body:
            msg += f": {body[:500]}"
        raise ShimHTTPError(r.status_code, msg)

    def healthcheck(self) -> Optional[dict]:
        try:
            r = self.c.get("/api/healthcheck", timeout=5)
            return r.json() if r.status_code == 200 else None
        except httpx.HTTPError:
            return None

    def host_info(self) -> dict:
        r = self.c.get("/api/host_info")
        r.raise_for_status()
        return r.json()

    def submit_task(self, task: dict) -> dict:
        """Submit (idempotent: 409 = the task already exists, its current state is returned)."""
        r = self._request("POST", "/api/tasks", json=task)
        if r.status_code == 409:
            return self.get_task(task["id"])
        self._raise_for_status(r)
        return r.json()

    def get_task(self, task_id: str) -> Optional[dict]:
        r = self._request("GET", f"/api/tasks/{task_id}")
        if r.status_code == 404:
            return None
        self._raise_for_status(r)
        return r.json()

    def list_tasks(self) -> List[str]:
        r = self._request("GET", "/api/tasks")
        self._raise_for_status(r)
        return r.json().get("ids", [])

    def terminate_task(self, task_id: str, reason: str = "", message: str = "", timeout: int = 10) -> None:
        r = self._request("POST", f"/api/tasks/{task_id}/terminate",
                          json={"termination_reason": reason, "termination_message": message, "timeout": timeout},
                          timeout=timeout + 30)
        if r.status_code != 404:
            self._raise_for_status(r)

    def remove_task(self, task_id: str) -> None:
        r = self._request("POST", f"/api/tasks/{task_id}/remove")
        if r.status_code not in (404, 409):
            self._raise_for_status(r)

    def gpu_health(self) -> Optional[dict]:
        """The shim's latest HIP health-probe state ``{state, started_at_ms, ran_at_ms, result}``
        (None: an API-1 shim, which has no probe endpoint)."""
        if self.api_version < 2:
            return None
        r = self._request("GET", "/api/gpu_health", timeout=5)
        if r.status_code == 404:
            return None
        self._raise_for_status(r)
        return r.json()

    def start_gpu_probe(self) -> str:
        """Ask the shim to (re-)run the probe off the job path: started | running | busy | unavailable."""
        if self.api_version < 2:
            return "unavailable"
        r = self._request("POST", "/api/gpu_health/probe", timeout=5)
        if r.status_code == 404:
            return "unavailable"
        return (r.json() or {}).get("state", "unavailable")


class RunnerClient:
    def __init__(self, base_url: str, transport: Optional[httpx.BaseTransport] = None):
        self.base_url = base_url
        self.c = _client(base_url, transport)

    def healthcheck(self) -> Optional[dict]:
        try:
            r = self.c.get("/api/healthcheck", timeout=5)
            return r.json() if r.status_code == 200 else None
        except httpx.HTTPError:
            return None

    def get_metrics(self) -> Optional[dict]:
        try:
            r = self.c.get("/api/metrics", timeout=10)
            return r.json() if r.status_code == 200 else None
        except httpx.HTTPError:
            return None

    def submit_job(self, run_spec: RunSpec, run_name: str, repo_data: Optional[dict], job_spec: JobSpec,
                   cluster_info: ClusterInfo, secrets: Dict[str, str], repo_credentials: Optional[dict]) -> None:
        body = {
            "run_spec": {
                "run_name": run_name, "repo_id": run_spec.repo_id,
                "repo_data": repo_data or {"repo_type": "virtual"},
                "configuration_path": run_spec.configuration_path,
            },
            "job_spec": json.loads(job_spec.model_dump_json()),
            "cluster_info": cluster_info.model_dump(mode="json"),
            "secrets": secrets,
            "repo_credentials": repo_credentials,
        }
        r = self.c.post("/api/submit", json=body)
        if r.status_code not in (200, 409):
            raise RunnerError(f"runner submit failed: {r.status_code} {r.text}")

    def upload_code(self, blob: bytes) -> None:
        r = self.c.post("/api/upload_code", content=blob, headers={"Content-Type": "application/octet-stream"})
        if r.status_code not in (200, 409):
            raise RunnerError(f"upload_code failed: {r.text}")

    def run_job(self) -> None:
        r = self.c.post("/api/run")
        if r.status_code not in (200, 409):
            raise RunnerError(f"run failed: {r.text}")

    def pull(self, timestamp: int, wait_ms: int = 0) -> dict:
        r = self.c.get("/api/pull", params={"timestamp": timestamp, "wait_ms": wait_ms},
                       timeout=REQUEST_TIMEOUT + wait_ms / 1000)
        r.raise_for_status()
        return r.json()

    def stop(self) -> None:
        try:
            self.c.post("/api/stop", timeout=5)
        except httpx.HTTPError:
            pass


# ---------------------------------------------------------------------------------------------
# reaching the agents
# ---------------------------------------------------------------------------------------------
def _ssh_target(jpd: JobProvisioningData) -> SSHTarget:
    proxy = None
    if jpd.ssh_proxy is not None:
        proxy = SSHTarget(jpd.ssh_proxy.hostname, jpd.ssh_proxy.username, jpd.ssh_proxy.port)
    return SSHTarget(jpd.hostname or "", jpd.username, jpd.ssh_port or 22, proxy)


def _is_direct(jpd: JobProvisioningData) -> bool:
    if jpd.backend == BackendType.LOCAL:
        return True
    data = json.loads(jpd.backend_data) if jpd.backend_data else {}
    return bool(data.get("direct"))  # trusted on-prem LAN: talk HTTP directly, no SSH


def shim_base_url(jpd: JobProvisioningData, private_key: str) -> str:
    data = json.loads(jpd.backend_data) if jpd.backend_data else {}
    port = int(data.get("shim_port") or DSTACK_SHIM_HTTP_PORT)
    if _is_direct(jpd):
        return f"http://{jpd.hostname or '127.0.0.1'}:{port}"
    local = get_tunnel_pool().forward(_ssh_target(jpd), private_key, port)
    return f"http://127.0.0.1:{local}"


def runner_base_url(jpd: JobProvisioningData, jrd: Optional[JobRuntimeData], private_key: str) -> str:
    port = DSTACK_RUNNER_HTTP_PORT
    if jrd is not None and jrd.ports:
        port = int(jrd.ports.get(DSTACK_RUNNER_HTTP_PORT, jrd.ports.get(str(DSTACK_RUNNER_HTTP_PORT), port)))
    return port_base_url(jpd, private_key, port)


def port_base_url(jpd: JobProvisioningData, private_key: str, port: int) -> str:
    """URL of ``port`` on the job's host: direct for local/LAN hosts, else a pooled SSH forward."""
    if _is_direct(jpd):
        return f"http://{jpd.hostname or '127.0.0.1'}:{port}"
    local = get_tunnel_pool().forward(_ssh_target(jpd), private_key, port)
    return f"http://127.0.0.1:{local}"


def get_shim_client(jpd: JobProvisioningData, private_key: str) -> ShimClient:
    return ShimClient(shim_base_url(jpd, private_key))


def get_runner_client(jpd: JobProvisioningData, jrd: Optional[JobRuntimeData], private_key: str) -> RunnerClient:
    return RunnerClient(runner_base_url(jpd, jrd, private_key))


__all__ = ["ShimClient", "ShimHTTPError", "RunnerClient", "parse_version", "get_shim_client", "get_runner_client", "port_base_url", "SSHError"]
