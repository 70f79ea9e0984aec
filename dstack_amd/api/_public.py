"""High-level Python API (reference: ``api/_public/__init__.py:17-95``, ``api/_public/runs.py:53-700``,
``api/_public/repos.py``).

``Client.from_config()`` -> ``client.runs.apply_configuration(conf, repo)`` -> ``Run`` with
``logs()`` / ``wait()`` / ``attach()`` / ``stop()``.  Logs are read from the server's log storage
(``/logs/poll``) while detached and, once attached, streamed straight from the runner's
``/logs_ws`` websocket through the SSH forward (lower latency for ``dstack apply``).
"""

from __future__ import annotations

import base64
import io
import os
import time
from typing import Dict, Iterator, List, Optional

from dstack_amd.api.server import APIClient, client_from_env_or_config
from dstack_amd.core.errors import ClientError, ConfigurationError, ResourceNotExistsError
from dstack_amd.core.models.configurations import AnyRunConfiguration, ServiceConfiguration
from dstack_amd.core.models.fleets import Fleet, FleetConfiguration, FleetSpec
from dstack_amd.core.models.profiles import Profile
from dstack_amd.core.models.repos import Repo, VirtualRepo
from dstack_amd.core.models.runs import JobStatus, Run as RunModel, RunPlan, RunSpec, RunStatus
from dstack_amd.core.models.volumes import Volume, VolumeConfiguration


class Run:
    def __init__(self, api: APIClient, project: str, run: RunModel, ssh_identity_file: Optional[str] = None):
        self._api = api
        self._project = project
        self._run = run
        self._ssh_identity_file = ssh_identity_file
        self._attach = None

    # ---- properties ---------------------------------------------------------------------------
    @property
    def name(self) -> str:
        return self._run.run_spec.run_name

    @property
    def status(self) -> RunStatus:
        return self._run.status

    @property
    def model(self) -> RunModel:
        return self._run

    @property
    def hostname(self) -> Optional[str]:
        jpd = self._latest_submission().job_provisioning_data if self._run.jobs else None
        return jpd.hostname if jpd else None

    @property
    def backend(self):
        jpd = self._latest_submission().job_provisioning_data if self._run.jobs else None
        return jpd.backend if jpd else None

    @property
    def ports(self) -> Optional[Dict[int, int]]:
        return self._attach.ports if self._attach else None

    @property
    def service_url(self) -> Optional[str]:
        if not isinstance(self._run.run_spec.configuration, ServiceConfiguration):
            return None
        if self._run.service is not None:
            url = self._run.service.url
            return url if url.startswith("http") else self._api.base_url + url
        return f"{self._api.base_url}/proxy/services/{self._project}/{self.name}/"

    @property
    def service_model(self) -> Optional["ServiceModel"]:
        """The OpenAI-compatible model a service publishes (``model:`` in its configuration): its
        name and the base URL of the model endpoint (in-server ``/proxy/models/<project>`` or the
        gateway's)."""
        if not isinstance(self._run.run_spec.configuration, ServiceConfiguration):
            raise ValueError("The run is not a service")
        svc = self._run.service
        if svc is None or svc.model is None:
            return None
        url = svc.model.base_url
        return ServiceModel(svc.model.name, url if url.startswith("http") else self._api.base_url + url)

    def _latest_submission(self, replica_num: int = 0, job_num: int = 0):
        for j in self._run.jobs:
            if j.job_spec.replica_num == replica_num and j.job_spec.job_num == job_num:
                return j.job_submissions[-1]
        return self._run.jobs[0].job_submissions[-1]

    # ---- lifecycle ----------------------------------------------------------------------------
    def refresh(self) -> "Run":
        self._run = self._api.runs.get(self._project, self.name)
        return self

    def stop(self, abort: bool = False):
        self._api.runs.stop(self._project, [self.name], abort)

    def wait(self, statuses=None, timeout: Optional[float] = None, poll: float = 0.25) -> RunStatus:
        """Block until the run reaches one of ``statuses`` (default: finished)."""
        deadline = None if timeout is None else time.time() + timeout
        while True:
            self.refresh()
            st = self.status
            if (statuses is None and st.is_finished()) or (statuses is not None and st in statuses):
                return st
            if deadline is not None and time.time() > deadline:
                raise TimeoutError(f"run {self.name} still {st.value} after {timeout}s")
            time.sleep(poll)

    def logs(self, start_time=None, diagnose: bool = False, replica_num: int = 0, job_num: int = 0,
             follow: bool = False, poll: float = 0.5) -> Iterator[bytes]:
        """Yield the job's log chunks; with ``follow`` keep yielding until the run finishes."""
        next_token = None
        while True:
            if not self._run.jobs:
                if not follow:
                    return
                time.sleep(poll)
                self.refresh()
                continue
            sub = self._latest_submission(replica_num, job_num)
            rewrite = None if diagnose else self._url_replacer(replica_num, job_num)
            while True:
                resp = self._api.logs.poll(self._project, self.name, sub.id, start_time=start_time,
                                           diagnose=diagnose, next_token=next_token)
                for ev in resp.logs:
                    chunk = base64.b64decode(ev.message)
                    yield rewrite(chunk) if rewrite else chunk
                if resp.next_token and resp.logs:
                    next_token = resp.next_token
                    continue
                break
            if not follow:
                return
            finished = self._run.status.is_finished()
            if finished:
                return
            time.sleep(poll)
            self.refresh()
            if self._run.status.is_finished():
                finished = True  # one more drain pass after termination

    def _url_replacer(self, replica_num: int = 0, job_num: int = 0):
        """Rewrites the container URLs a job prints: to the forwarded local ports when attached,
        to the service's public URL for a service (``core.services.logs.URLReplacer``)."""
        import urllib.parse

        from dstack_amd.core.services.logs import URLReplacer

        job = next((j for j in self._run.jobs if j.job_spec.replica_num == replica_num
                    and j.job_spec.job_num == job_num), self._run.jobs[0] if self._run.jobs else None)
        if job is None:
            return None
        conf = self._run.run_spec.configuration
        if self.ports:
            jpd = job.job_submissions[-1].job_provisioning_data
            return URLReplacer(ports=self.ports, app_specs=job.job_spec.app_specs or [], hostname="127.0.0.1",
                               secure=False, ip_address=jpd.hostname if jpd else None)
        if isinstance(conf, ServiceConfiguration) and self.service_url:
            u = urllib.parse.urlsplit(self.service_url)
            secure = u.scheme == "https"
            return URLReplacer(ports={conf.port.container_port: u.port or (443 if secure else 80)}, app_specs=[],
                               hostname=u.hostname or "", secure=secure, path_prefix=u.path if u.path != "/" else "")
        return None

    def attach(self, ssh_identity_file: Optional[str] = None, bind_address: str = "127.0.0.1",
               ports_overrides: Optional[Dict[int, int]] = None) -> bool:
        """Forward the job's ports to localhost (and for remote hosts open an SSH master)."""
        from dstack_amd.core.services.ssh.attach import RunAttach

        self.refresh()
        sub = self._latest_submission()
        if sub.status not in (JobStatus.RUNNING,):
            return False
        self._attach = RunAttach(self._run, sub, ssh_identity_file or self._ssh_identity_file,
                                 bind_address=bind_address, ports_overrides=ports_overrides or {})
        self._attach.open()
        return True

    def detach(self):
        if self._attach is not None:
            self._attach.close()
            self._attach = None

    def __repr__(self) -> str:
        return f"<Run '{self.name}' {self.status.value}>"


class ServiceModel:
    def __init__(self, name: str, url: str):
        self.name = name
        self.url = url

    def __repr__(self) -> str:
        return f"<ServiceModel {self.name!r}>"


class RunCollection:
    def __init__(self, api: APIClient, project: str, client: "Client"):
        self._api = api
        self._project = project
        self._client = client

    def get_offers(self, profile, requirements):
        """Offers (pool instances and backends) for a profile + requirements pair."""
        return self._api.pool.get_offers(self._project, profile, requirements)

    def create_instance(self, profile, requirements):
        """Provision an instance from the best offer without a run (``dstack pool add``)."""
        return self._api.pool.create_instance(self._project, profile, requirements)

    def _upload(self, repo: Repo) -> Optional[str]:
        buf = io.BytesIO()
        h = repo.write_code_file(buf)
        data = buf.getvalue()
        if not data:
            return h
        return self._api.repos.upload_code(self._project, repo.repo_id, data)

    def get_plan(self, configuration: AnyRunConfiguration, repo: Optional[Repo] = None,
                 configuration_path: Optional[str] = None, profile: Optional[Profile] = None,
                 run_name: Optional[str] = None, ssh_identity_file: Optional[str] = None,
                 max_offers: Optional[int] = None) -> RunPlan:
        repo = repo or VirtualRepo()
        self._client.repos.init(repo)
        code_hash = self._upload(repo)
        pub = ""
        key = ssh_identity_file or self._client.ssh_identity_file
        if key and os.path.exists(str(key) + ".pub"):
            with open(str(key) + ".pub") as f:
                pub = f.read().strip()
        spec = RunSpec(run_name=run_name or getattr(configuration, "name", None), repo_id=repo.repo_id,
                       repo_data=repo.run_repo_data, repo_code_hash=code_hash,
                       working_dir=getattr(configuration, "working_dir", None),
                       configuration_path=configuration_path, configuration=configuration, profile=profile,
                       ssh_key_pub=pub)
        return self._api.runs.get_plan(self._project, spec, max_offers)

    def exec_plan(self, plan: RunPlan, repo: Optional[Repo] = None, force: bool = False) -> Run:
        run = self._api.runs.apply_plan(self._project, plan, force=force)
        return Run(self._api, self._project, run, self._client.ssh_identity_file)

    def apply_configuration(self, configuration: AnyRunConfiguration, repo: Optional[Repo] = None,
                            configuration_path: Optional[str] = None, profile: Optional[Profile] = None,
                            run_name: Optional[str] = None, force: bool = False) -> Run:
        plan = self.get_plan(configuration, repo, configuration_path, profile, run_name)
        return self.exec_plan(plan, repo, force=force)

    def submit(self, configuration: AnyRunConfiguration, repo: Optional[Repo] = None,
               run_name: Optional[str] = None, profile: Optional[Profile] = None) -> Run:
        repo = repo or VirtualRepo()
        self._client.repos.init(repo)
        code_hash = self._upload(repo)
        spec = RunSpec(run_name=run_name or getattr(configuration, "name", None), repo_id=repo.repo_id,
                       repo_data=repo.run_repo_data, repo_code_hash=code_hash, configuration=configuration,
                       profile=profile)
        return Run(self._api, self._project, self._api.runs.submit(self._project, spec),
                   self._client.ssh_identity_file)

    def list(self, all: bool = False, limit: int = 100) -> List[Run]:
        runs = self._api.runs.list(self._project, only_active=not all, limit=limit)
        return [Run(self._api, self._project, r, self._client.ssh_identity_file) for r in runs]

    def get(self, run_name: str) -> Optional[Run]:
        try:
            return Run(self._api, self._project, self._api.runs.get(self._project, run_name),
                       self._client.ssh_identity_file)
        except (ClientError, ResourceNotExistsError):
            return None


class RepoCollection:
    def __init__(self, api: APIClient, project: str):
        self._api = api
        self._project = project
        self._inited: set = set()

    def init(self, repo: Repo, git_identity_file: Optional[str] = None, oauth_token: Optional[str] = None):
        if repo.repo_id in self._inited:
            return
        creds = None
        if git_identity_file or oauth_token:
            creds = {"protocol": "ssh" if git_identity_file else "https", "oauth_token": oauth_token,
                     "private_key": open(git_identity_file).read() if git_identity_file else None}
        info = repo.get_repo_info().model_dump(mode="json")
        self._api.repos.init(self._project, repo.repo_id, info, creds)
        self._inited.add(repo.repo_id)

    def is_initialized(self, repo: Repo) -> bool:
        try:
            self._api.repos.get(self._project, repo.repo_id)
            return True
        except Exception:  # noqa: BLE001
            return False

    def load(self, repo_dir: str, local: bool = False, init: bool = False,
             git_identity_file: Optional[str] = None, oauth_token: Optional[str] = None) -> Repo:
        """The repo of a local directory (reference ``RepoCollection.load``).

        ``init=False``: the directory must have been initialised (``dstack init`` or
        ``load(..., init=True)``), both in the CLI config and on the server.  ``init=True``: a git
        checkout with a remote becomes a ``RemoteRepo`` (unless ``local``), anything else a
        ``LocalRepo``; it is initialised in the project and recorded in the CLI config."""
        from dstack_amd.core.errors import ConfigurationError
        from dstack_amd.core.models.repos import LocalRepo, RemoteRepo
        from dstack_amd.core.services.configs import ConfigManager

        cm = ConfigManager()
        hint = "The repo is not initialized. Run `dstack init` in it or load it with init=True."
        if not init:
            rc = cm.get_repo_config(repo_dir)
            if rc is None:
                raise ConfigurationError(hint)
            repo = LocalRepo(repo_dir, rc.repo_id) if rc.repo_type == "local" else RemoteRepo(repo_dir,
                                                                                              repo_id=rc.repo_id)
            if not self.is_initialized(repo):
                raise ConfigurationError(hint)
            return repo
        repo: Repo = LocalRepo(repo_dir)
        if not local:
            try:
                repo = RemoteRepo(repo_dir)
            except Exception:  # noqa: BLE001 - not a git checkout, or no remote: upload the tree
                repo = LocalRepo(repo_dir)
        self.init(repo, git_identity_file, oauth_token)
        key = git_identity_file or str(cm.ensure_ssh_key())
        cm.save_repo_config(repo_dir, repo.repo_id, "local" if isinstance(repo, LocalRepo) else "remote", key)
        return repo


class FleetCollection:
    def __init__(self, api: APIClient, project: str):
        self._api, self._project = api, project

    def apply_configuration(self, configuration: FleetConfiguration) -> Fleet:
        spec = FleetSpec(configuration=configuration)
        return self._api.fleets.create(self._project, spec)

    def list(self) -> List[Fleet]:
        return self._api.fleets.list(self._project)

    def get(self, name: str) -> Fleet:
        return self._api.fleets.get(self._project, name)

    def delete(self, name: str):
        self._api.fleets.delete(self._project, [name])


class VolumeCollection:
    def __init__(self, api: APIClient, project: str):
        self._api, self._project = api, project

    def create(self, configuration: VolumeConfiguration) -> Volume:
        return self._api.volumes.create(self._project, configuration)

    def list(self) -> List[Volume]:
        return self._api.volumes.list(self._project)

    def get(self, name: str) -> Volume:
        return self._api.volumes.get(self._project, name)

    def delete(self, name: str):
        self._api.volumes.delete(self._project, [name])


class Backend:
    """A backend configured in the project (reference: ``dstack/api/_public/backends.py``)."""

    def __init__(self, api: APIClient, info):
        self._api = api
        self._info = info

    @property
    def name(self) -> str:
        return self._info.name.value if hasattr(self._info.name, "value") else str(self._info.name)

    @property
    def config(self) -> dict:
        """Settings without credentials."""
        return dict(self._info.config)

    def __repr__(self) -> str:
        return f"<Backend '{self.name}'>"


class BackendCollection:
    def __init__(self, api: APIClient, project: str):
        self._api, self._project = api, project

    def list(self) -> List[Backend]:
        return [Backend(self._api, b) for b in self._api.projects.get(self._project).backends]

    def create(self, config: dict) -> Backend:
        """``config`` is a ``projects[].backends[]`` mapping of the server config (type, creds, ...)."""
        self._api.backends.create(self._project, config)
        return next(b for b in self.list() if b.name == config["type"])

    def delete(self, names: List[str]):
        self._api.backends.delete(self._project, names)


class PoolInstance:
    """One pool of the deprecated pools API (reference ``api/_public/pools.py``)."""

    def __init__(self, api_client: APIClient, pool):
        self._api = api_client
        self._pool = pool

    @property
    def name(self) -> str:
        return self._pool.name

    @property
    def default(self) -> bool:
        return self._pool.default

    @property
    def total_instances(self) -> int:
        return self._pool.total_instances

    @property
    def available_instances(self) -> int:
        return self._pool.available_instances

    def __repr__(self) -> str:
        return f"<PoolInstance '{self.name}'>"

    __str__ = __repr__


class PoolCollection:
    """Operations with pools (deprecated in the reference in favour of fleets; kept so old scripts
    using ``client.pool`` keep working)."""

    def __init__(self, api_client: APIClient, project_name: str):
        self._api = api_client
        self._project = project_name

    def list(self) -> List[PoolInstance]:
        return [PoolInstance(self._api, p) for p in self._api.pool.list(self._project)]

    def show(self, name: Optional[str] = None):
        """The pool's instances (``None``: the project's default pool)."""
        return self._api.pool.show(self._project, name)

    def create(self, name: str) -> PoolInstance:
        self._api.pool.create(self._project, name)
        return next(p for p in self.list() if p.name == name)

    def delete(self, name: str, force: bool = False):
        self._api.pool.delete(self._project, name, force)


class Client:
    def __init__(self, api_client: APIClient, project_name: str, ssh_identity_file: Optional[str] = None):
        self.api = api_client
        self.project = project_name
        self.ssh_identity_file = ssh_identity_file
        self.repos = RepoCollection(api_client, project_name)
        self.runs = RunCollection(api_client, project_name, self)
        self.fleets = FleetCollection(api_client, project_name)
        self.volumes = VolumeCollection(api_client, project_name)
        self.backends = BackendCollection(api_client, project_name)
        self.pool = PoolCollection(api_client, project_name)

    @staticmethod
    def from_config(project_name: Optional[str] = None, server_url: Optional[str] = None,
                    user_token: Optional[str] = None, ssh_identity_file: Optional[str] = None) -> "Client":
        if server_url and user_token:
            api, project = APIClient(server_url, user_token), project_name or "main"
        elif server_url or user_token:
            raise ConfigurationError("server_url and user_token must be given together")
        else:
            api, project = client_from_env_or_config(project_name)
        if ssh_identity_file is None:
            try:
                from dstack_amd.core.services.configs import ConfigManager

                ssh_identity_file = str(ConfigManager().ensure_ssh_key())
            except Exception:  # noqa: BLE001 - ssh-keygen missing: attach just won't work
                ssh_identity_file = None
        return Client(api, project, ssh_identity_file)
