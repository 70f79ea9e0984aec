"""Low-level REST client (reference: ``api/server/__init__.py:44-186`` and the per-resource
groups ``api/server/_*.py``).  Every endpoint is a JSON ``POST``; responses are parsed into the
``core.models`` pydantic types.  One pooled ``httpx.Client`` (keep-alive) per APIClient — the
CLI's ``dstack apply`` issues a handful of calls and the cold-start bench hundreds.
"""

from __future__ import annotations

import os
import time
from datetime import datetime
from typing import Any, Dict, List, Optional, Type, TypeVar, Union
from uuid import UUID

import httpx
from pydantic import BaseModel, TypeAdapter

from dstack_amd import __version__
from dstack_amd.core.errors import (
    ClientError,
    ResourceExistsError,
    ResourceNotExistsError,
    ServerClientError,
    ServerClientErrorCode,
    URLNotFoundError,
)
from dstack_amd.core.models.fleets import Fleet, FleetPlan, FleetSpec, Instance, Pool, PoolInstances
from dstack_amd.core.models.instances import SSHKey
from dstack_amd.core.models.profiles import Profile
from dstack_amd.core.models.gateways import Gateway, GatewayConfiguration
from dstack_amd.core.models.logs import JobMetrics, JobSubmissionLogs
from dstack_amd.core.models.repos import RepoHead
from dstack_amd.core.models.runs import ApplyRunPlanInput, PoolInstanceOffers, Requirements, Run, RunPlan, RunSpec
from dstack_amd.core.models.users import Project, ServerInfo, User, UserWithCreds
from dstack_amd.core.models.volumes import Volume, VolumeConfiguration

T = TypeVar("T")


def _dump(v: Any) -> Any:
    if isinstance(v, BaseModel):
        return v.model_dump(mode="json", exclude_none=False)
    if isinstance(v, dict):
        return {k: _dump(x) for k, x in v.items() if x is not None}
    if isinstance(v, (list, tuple)):
        return [_dump(x) for x in v]
    if isinstance(v, (UUID, datetime)):
        return str(v) if isinstance(v, UUID) else v.isoformat()
    return v


class APIClient:
    def __init__(self, base_url: str, token: str, timeout: float = 60.0):
        self.base_url = base_url.rstrip("/")
        self.token = token
        self._http = httpx.Client(base_url=self.base_url, timeout=timeout, headers={
            "Authorization": f"Bearer {token}", "X-API-VERSION": __version__,
            "User-Agent": f"dstack-amd/{__version__}"})
        self.server = _Server(self)
        self.users = _Users(self)
        self.projects = _Projects(self)
        self.backends = _Backends(self)
        self.secrets = _Secrets(self)
        self.repos = _Repos(self)
        self.runs = _Runs(self)
        self.logs = _Logs(self)
        self.metrics = _Metrics(self)
        self.fleets = _Fleets(self)
        self.instances = _Instances(self)
        self.volumes = _Volumes(self)
        self.gateways = _Gateways(self)
        self.pool = _Pool(self)

    def close(self):
        self._http.close()

    def _request(self, path: str, body: Any = None, method: str = "POST", raw: Optional[bytes] = None,
                 params: Optional[Dict[str, Any]] = None, retries: int = 3) -> httpx.Response:
        for attempt in range(retries):
            try:
                if raw is not None:
                    r = self._http.request(method, path, content=raw, params=params,
                                           headers={"content-type": "application/octet-stream"})
                elif method == "GET":
                    r = self._http.get(path, params=params)
                else:
                    r = self._http.request(method, path, json=_dump(body) if body is not None else {}, params=params)
                break
            except httpx.TransportError as e:
                if attempt == retries - 1:
                    raise ClientError(f"Cannot connect to the dstack server at {self.base_url}: {e}") from e
                time.sleep(0.2 * (attempt + 1))
        if r.status_code == 404:
            raise URLNotFoundError(f"{method} {path}: not found")
        if r.status_code in (400, 401, 403, 422):
            raise _server_error(r)
        r.raise_for_status()
        return r

    def post(self, path: str, body: Any = None, model: Optional[Type[T]] = None, **kw) -> Any:
        r = self._request(path, body, **kw)
        data = r.json() if r.content else None
        if model is None:
            return data
        return TypeAdapter(model).validate_python(data)


def _server_error(r: httpx.Response) -> ServerClientError:
    try:
        detail = r.json().get("detail")
    except ValueError:
        return ServerClientError(r.text or f"HTTP {r.status_code}")
    if isinstance(detail, list) and detail:
        msgs = []
        for d in detail:
            loc = d.get("loc")
            msgs.append(f"{'.'.join(str(x) for x in loc[1:])}: {d['msg']}" if loc else d.get("msg", ""))
        code = detail[0].get("code", "error")
        cls = {ServerClientErrorCode.RESOURCE_NOT_EXISTS: ResourceNotExistsError,
               ServerClientErrorCode.RESOURCE_EXISTS: ResourceExistsError}.get(code, ServerClientError)
        e = cls("; ".join(msgs))
        e.code = code
        return e
    e = ServerClientError(str(detail))
    return e


class _Group:
    def __init__(self, c: APIClient):
        self._c = c


class _Server(_Group):
    def get_info(self) -> ServerInfo:
        return self._c.post("/api/server/get_info", model=ServerInfo)


class _Users(_Group):
    def list(self) -> List[User]:
        return self._c.post("/api/users/list", model=List[User])

    def get_my_user(self) -> UserWithCreds:
        return self._c.post("/api/users/get_my_user", model=UserWithCreds)

    def get_user(self, username: str) -> UserWithCreds:
        return self._c.post("/api/users/get_user", {"username": username}, model=UserWithCreds)

    def create(self, username: str, global_role: str = "user", email: Optional[str] = None,
               active: bool = True) -> UserWithCreds:
        return self._c.post("/api/users/create", {"username": username, "global_role": global_role, "email": email,
                                                  "active": active}, model=UserWithCreds)

    def update(self, username: str, global_role: str, email: Optional[str] = None, active: bool = True) -> User:
        return self._c.post("/api/users/update", {"username": username, "global_role": global_role, "email": email,
                                                  "active": active}, model=User)

    def refresh_token(self, username: str) -> UserWithCreds:
        return self._c.post("/api/users/refresh_token", {"username": username}, model=UserWithCreds)

    def delete(self, users: List[str]):
        self._c.post("/api/users/delete", {"users": users})


class _Projects(_Group):
    def list(self) -> List[Project]:
        return self._c.post("/api/projects/list", model=List[Project])

    def create(self, project_name: str) -> Project:
        return self._c.post("/api/projects/create", {"project_name": project_name}, model=Project)

    def delete(self, projects_names: List[str]):
        self._c.post("/api/projects/delete", {"projects_names": projects_names})

    def get(self, project_name: str) -> Project:
        return self._c.post(f"/api/projects/{project_name}/get", model=Project)

    def set_members(self, project_name: str, members: List[Dict[str, str]]) -> Project:
        return self._c.post(f"/api/projects/{project_name}/set_members", {"members": members}, model=Project)


class _Backends(_Group):
    def list_types(self) -> List[str]:
        return self._c.post("/api/backends/list_types")

    def create(self, project_name: str, config: dict) -> dict:
        return self._c.post(f"/api/project/{project_name}/backends/create", config)

    def update(self, project_name: str, config: dict) -> dict:
        return self._c.post(f"/api/project/{project_name}/backends/update", config)

    def config_info(self, project_name: str, backend_name: str) -> dict:
        return self._c.post(f"/api/project/{project_name}/backends/{backend_name}/config_info")

    def create_yaml(self, project_name: str, config_yaml: str):
        self._c.post(f"/api/project/{project_name}/backends/create_yaml", {"config_yaml": config_yaml})

    def update_yaml(self, project_name: str, config_yaml: str):
        self._c.post(f"/api/project/{project_name}/backends/update_yaml", {"config_yaml": config_yaml})

    def get_yaml(self, project_name: str, backend_name: str) -> dict:
        return self._c.post(f"/api/project/{project_name}/backends/{backend_name}/get_yaml")

    def delete(self, project_name: str, backends_names: List[str]):
        self._c.post(f"/api/project/{project_name}/backends/delete", {"backends_names": backends_names})


class _Secrets(_Group):
    def list(self, project_name: str) -> list:
        return self._c.post(f"/api/project/{project_name}/secrets/list")

    def get(self, project_name: str, name: str) -> dict:
        return self._c.post(f"/api/project/{project_name}/secrets/get", {"name": name})

    def create_or_update(self, project_name: str, name: str, value: str) -> dict:
        return self._c.post(f"/api/project/{project_name}/secrets/add", {"name": name, "value": value})

    def delete(self, project_name: str, names: List[str]):
        self._c.post(f"/api/project/{project_name}/secrets/delete", {"secrets_names": names})


class _Repos(_Group):
    def list(self, project_name: str) -> List[RepoHead]:
        return self._c.post(f"/api/project/{project_name}/repos/list", model=List[RepoHead])

    def get(self, project_name: str, repo_id: str, include_creds: bool = False) -> dict:
        return self._c.post(f"/api/project/{project_name}/repos/get",
                            {"repo_id": repo_id, "include_creds": include_creds})

    def init(self, project_name: str, repo_id: str, repo_info: dict, repo_creds: Optional[dict] = None):
        self._c.post(f"/api/project/{project_name}/repos/init",
                     {"repo_id": repo_id, "repo_info": repo_info, "repo_creds": repo_creds})

    def delete(self, project_name: str, repos_ids: List[str]):
        self._c.post(f"/api/project/{project_name}/repos/delete", {"repos_ids": repos_ids})

    def upload_code(self, project_name: str, repo_id: str, blob: bytes) -> str:
        r = self._c._request(f"/api/project/{project_name}/repos/upload_code", raw=blob, params={"repo_id": repo_id})
        return r.json()["blob_hash"]


class _Runs(_Group):
    def list(self, project_name: Optional[str] = None, repo_id: Optional[str] = None, only_active: bool = False,
             limit: int = 100, prev_submitted_at: Optional[datetime] = None, prev_run_id: Optional[UUID] = None,
             username: Optional[str] = None) -> List[Run]:
        return self._c.post("/api/runs/list", {
            "project_name": project_name, "repo_id": repo_id, "only_active": only_active, "limit": limit,
            "prev_submitted_at": prev_submitted_at, "prev_run_id": prev_run_id, "username": username}, model=List[Run])

    def get(self, project_name: str, run_name: str) -> Run:
        return self._c.post(f"/api/project/{project_name}/runs/get", {"run_name": run_name}, model=Run)

    def get_plan(self, project_name: str, run_spec: RunSpec, max_offers: Optional[int] = None) -> RunPlan:
        return self._c.post(f"/api/project/{project_name}/runs/get_plan",
                            {"run_spec": run_spec, "max_offers": max_offers}, model=RunPlan)

    def apply_plan(self, project_name: str, plan: Union[RunPlan, ApplyRunPlanInput], force: bool = False) -> Run:
        inp = ApplyRunPlanInput(run_spec=plan.run_spec, current_resource=plan.current_resource)
        return self._c.post(f"/api/project/{project_name}/runs/apply", {"plan": inp, "force": force}, model=Run)

    def submit(self, project_name: str, run_spec: RunSpec) -> Run:
        return self._c.post(f"/api/project/{project_name}/runs/submit", {"run_spec": run_spec}, model=Run)

    def stop(self, project_name: str, runs_names: List[str], abort: bool = False):
        self._c.post(f"/api/project/{project_name}/runs/stop", {"runs_names": runs_names, "abort": abort})

    def delete(self, project_name: str, runs_names: List[str]):
        self._c.post(f"/api/project/{project_name}/runs/delete", {"runs_names": runs_names})


class _Logs(_Group):
    def poll(self, project_name: str, run_name: str, job_submission_id, start_time: Optional[datetime] = None,
             end_time: Optional[datetime] = None, descending: bool = False, limit: int = 1000,
             diagnose: bool = False, next_token: Optional[str] = None) -> JobSubmissionLogs:
        return self._c.post(f"/api/project/{project_name}/logs/poll", {
            "run_name": run_name, "job_submission_id": str(job_submission_id), "start_time": start_time,
            "end_time": end_time, "descending": descending, "limit": limit, "diagnose": diagnose,
            "next_token": next_token}, model=JobSubmissionLogs)


class _Metrics(_Group):
    def get_job_metrics(self, project_name: str, run_name: str, replica_num: int = 0, job_num: int = 0,
                        limit: int = 2) -> JobMetrics:
        r = self._c._request(f"/api/project/{project_name}/metrics/job/{run_name}", method="GET",
                             params={"replica_num": replica_num, "job_num": job_num, "limit": limit})
        return JobMetrics.model_validate(r.json())


class _Fleets(_Group):
    def list(self, project_name: str) -> List[Fleet]:
        return self._c.post(f"/api/project/{project_name}/fleets/list", model=List[Fleet])

    def get(self, project_name: str, name: str) -> Fleet:
        return self._c.post(f"/api/project/{project_name}/fleets/get", {"name": name}, model=Fleet)

    def get_plan(self, project_name: str, spec: FleetSpec) -> FleetPlan:
        return self._c.post(f"/api/project/{project_name}/fleets/get_plan", {"spec": spec}, model=FleetPlan)

    def create(self, project_name: str, spec: FleetSpec) -> Fleet:
        return self._c.post(f"/api/project/{project_name}/fleets/create", {"spec": spec}, model=Fleet)

    def delete(self, project_name: str, names: List[str]):
        self._c.post(f"/api/project/{project_name}/fleets/delete", {"names": names})

    def delete_instances(self, project_name: str, name: str, instance_nums: List[int]):
        self._c.post(f"/api/project/{project_name}/fleets/delete_instances",
                     {"name": name, "instance_nums": instance_nums})


class _Instances(_Group):
    def list(self, project_names: Optional[List[str]] = None, only_active: bool = False) -> List[Instance]:
        return self._c.post("/api/instances/list", {"project_names": project_names, "only_active": only_active},
                            model=List[Instance])


class _Volumes(_Group):
    def list(self, project_name: str) -> List[Volume]:
        return self._c.post(f"/api/project/{project_name}/volumes/list", model=List[Volume])

    def get(self, project_name: str, name: str) -> Volume:
        return self._c.post(f"/api/project/{project_name}/volumes/get", {"name": name}, model=Volume)

    def create(self, project_name: str, configuration: VolumeConfiguration) -> Volume:
        return self._c.post(f"/api/project/{project_name}/volumes/create", {"configuration": configuration},
                            model=Volume)

    def delete(self, project_name: str, names: List[str]):
        self._c.post(f"/api/project/{project_name}/volumes/delete", {"names": names})


class _Gateways(_Group):
    def list(self, project_name: str) -> List[Gateway]:
        return self._c.post(f"/api/project/{project_name}/gateways/list", model=List[Gateway])

    def get(self, project_name: str, name: str) -> Gateway:
        return self._c.post(f"/api/project/{project_name}/gateways/get", {"name": name}, model=Gateway)

    def create(self, project_name: str, configuration: GatewayConfiguration) -> Gateway:
        return self._c.post(f"/api/project/{project_name}/gateways/create", {"configuration": configuration},
                            model=Gateway)

    def delete(self, project_name: str, names: List[str]):
        self._c.post(f"/api/project/{project_name}/gateways/delete", {"names": names})

    def set_default(self, project_name: str, name: str):
        self._c.post(f"/api/project/{project_name}/gateways/set_default", {"name": name})

    def set_wildcard_domain(self, project_name: str, name: str, wildcard_domain: Optional[str]) -> Gateway:
        return self._c.post(f"/api/project/{project_name}/gateways/set_wildcard_domain",
                            {"name": name, "wildcard_domain": wildcard_domain}, model=Gateway)


class _Pool(_Group):
    """Legacy pool API (deprecated in the reference in favour of fleets; kept for old clients)."""

    def list(self, project_name: str) -> List[Pool]:
        return self._c.post(f"/api/project/{project_name}/pool/list", model=List[Pool])

    def show(self, project_name: str, pool_name: Optional[str] = None) -> PoolInstances:
        return self._c.post(f"/api/project/{project_name}/pool/show", {"name": pool_name}, model=PoolInstances)

    def create(self, project_name: str, pool_name: str):
        self._c.post(f"/api/project/{project_name}/pool/create", {"name": pool_name})

    def delete(self, project_name: str, pool_name: str, force: bool = False):
        self._c.post(f"/api/project/{project_name}/pool/delete", {"name": pool_name, "force": force})

    def set_default(self, project_name: str, pool_name: str):
        self._c.post(f"/api/project/{project_name}/pool/set_default", {"pool_name": pool_name})

    def remove(self, project_name: str, pool_name: str, instance_name: str, force: bool = False):
        self._c.post(f"/api/project/{project_name}/pool/remove",
                     {"pool_name": pool_name, "instance_name": instance_name, "force": force})

    def add_remote(self, project_name: str, host: str, port: int, ssh_user: str, ssh_keys: List[SSHKey],
                   pool_name: Optional[str] = None, instance_name: Optional[str] = None,
                   region: Optional[str] = None, instance_network: Optional[str] = None) -> Instance:
        return self._c.post(f"/api/project/{project_name}/pool/add_remote", {
            "pool_name": pool_name, "instance_name": instance_name, "instance_network": instance_network,
            "region": region, "host": host, "port": port, "ssh_user": ssh_user,
            "ssh_keys": [_dump(k) for k in ssh_keys]}, model=Instance)

    def get_offers(self, project_name: str, profile: Profile, requirements: Requirements) -> PoolInstanceOffers:
        return self._c.post(f"/api/project/{project_name}/runs/get_offers",
                            {"profile": _dump(profile), "requirements": _dump(requirements)},
                            model=PoolInstanceOffers)

    def create_instance(self, project_name: str, profile: Profile, requirements: Requirements) -> Instance:
        return self._c.post(f"/api/project/{project_name}/runs/create_instance",
                            {"profile": _dump(profile), "requirements": _dump(requirements)}, model=Instance)


def client_from_env_or_config(project: Optional[str] = None) -> "tuple[APIClient, str]":
    """``DSTACK_SERVER_URL``/``DSTACK_TOKEN``/``DSTACK_PROJECT`` override ``~/.dstack/config.yml``."""
    url, token, name = os.getenv("DSTACK_SERVER_URL"), os.getenv("DSTACK_TOKEN"), project or os.getenv("DSTACK_PROJECT")
    if url and token:
        return APIClient(url, token), name or "main"
    from dstack_amd.core.services.configs import ConfigManager

    pc = ConfigManager().get_project_config(name)
    if pc is None:
        raise ClientError("No project configured: run `dstack config --url URL --token TOKEN --project NAME` "
                          "(or start `dstack server`, which configures the local project)")
    return APIClient(pc.url, pc.token), pc.name
