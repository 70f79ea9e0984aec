"""HTTP clients for the native agents (reference: ``S/services/runner/client.py:47-389``) and the
connection logic that reaches them: loopback for the ``local`` backend, pooled SSH port forwards
for remote hosts (``core/services/ssh/tunnel.py``)."""

from __future__ import annotations

import json
from typing import Any, Dict, List, Optional

import httpx

from dstack_amd.core.backends.base import DSTACK_RUNNER_HTTP_PORT, DSTACK_SHIM_HTTP_PORT
from dstack_amd.core.errors import RunnerError, SSHError
from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.runs import ClusterInfo, JobProvisioningData, JobRuntimeData, JobSpec, RunSpec
from dstack_amd.core.services.ssh.tunnel import SSHTarget, get_tunnel_pool

REQUEST_TIMEOUT = 15.0

_clients: Dict[str, httpx.Client] = {}


def _client(base_url: str) -> httpx.Client:
    c = _clients.get(base_url)
    if c is None:
        c = httpx.Client(base_url=base_url, timeout=REQUEST_TIMEOUT)
        _clients[base_url] = c
    return c


class ShimClient:
    def __init__(self, base_url: str):
        self.base_url = base_url
        self.c = _client(base_url)

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
        r = self.c.post("/api/tasks", json=task)
        if r.status_code == 409:
            return self.get_task(task["id"])
        if r.status_code != 200:
            raise RunnerError(f"shim submit failed: {r.status_code} {r.text}")
        return r.json()

    def get_task(self, task_id: str) -> Optional[dict]:
        r = self.c.get(f"/api/tasks/{task_id}")
        if r.status_code == 404:
            return None
        r.raise_for_status()
        return r.json()

    def list_tasks(self) -> List[str]:
        r = self.c.get("/api/tasks")
        r.raise_for_status()
        return r.json().get("ids", [])

    def terminate_task(self, task_id: str, reason: str = "", message: str = "", timeout: int = 10) -> None:
        r = self.c.post(f"/api/tasks/{task_id}/terminate",
                        json={"termination_reason": reason, "termination_message": message, "timeout": timeout},
                        timeout=timeout + 30)
        if r.status_code not in (200, 404):
            raise RunnerError(f"terminate failed: {r.text}")

    def remove_task(self, task_id: str) -> None:
        r = self.c.post(f"/api/tasks/{task_id}/remove")
        if r.status_code not in (200, 404, 409):
            raise RunnerError(f"remove failed: {r.text}")

    def gpu_health(self) -> Optional[dict]:
        """The shim's latest HIP health-probe state ``{state, started_at_ms, ran_at_ms, result}``
        (None: a shim without the endpoint)."""
        r = self.c.get("/api/gpu_health", timeout=5)
        if r.status_code == 404:
            return None
        r.raise_for_status()
        return r.json()

    def start_gpu_probe(self) -> str:
        """Ask the shim to (re-)run the probe off the job path: started | running | busy | unavailable."""
        r = self.c.post("/api/gpu_health/probe", timeout=5)
        if r.status_code == 404:
            return "unavailable"
        return (r.json() or {}).get("state", "unavailable")


class RunnerClient:
    def __init__(self, base_url: str):
        self.base_url = base_url
        self.c = _client(base_url)

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


__all__ = ["ShimClient", "RunnerClient", "get_shim_client", "get_runner_client", "port_base_url", "SSHError"]
