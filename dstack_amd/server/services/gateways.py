"""Gateways (reference: ``S/services/gateways/__init__.py:88-559``, ``client.py:16-190``).

A gateway is a host running ``dstack_amd.proxy.gateway`` (nginx + stats + OpenAI model proxy).
The server talks to its REST API (``/api/registry/...``, ``/api/stats``) — over an SSH tunnel for
cloud gateways, or directly for ``local``/on-prem gateways (``backend_data.direct``).
"""

from __future__ import annotations

import json
import logging
import uuid
from typing import List, Optional

import httpx
from sqlalchemy import select
from sqlalchemy.orm import Session

from dstack_amd.core.errors import GatewayError, ResourceExistsError, ResourceNotExistsError, ServerClientError
from dstack_amd.core.models.backends import (
    BACKENDS_WITH_GATEWAY_SUPPORT,
    BACKENDS_WITH_PRIVATE_GATEWAY_SUPPORT,
    BackendType,
)
from dstack_amd.core.models.gateways import (
    Gateway,
    GatewayConfiguration,
    GatewayPlan,
    GatewaySpec,
    GatewayStatus,
)
from dstack_amd.core.models.runs import RunSpec
from dstack_amd.server.background import scheduler
from dstack_amd.server.models import BackendModel, GatewayComputeModel, GatewayModel, JobModel, ProjectModel, RunModel, UserModel
from dstack_amd.server.services import jobs as jobs_services
from dstack_amd.utils.common import generate_name, generate_rsa_key_pair, get_current_datetime

logger = logging.getLogger(__name__)


def gateway_model_to_gateway(g: GatewayModel) -> Gateway:
    conf = GatewayConfiguration.model_validate_json(g.configuration) if g.configuration else \
        GatewayConfiguration(backend=BackendType(g.backend.type), region=g.region)
    comp = g.gateway_compute
    return Gateway(name=g.name, configuration=conf, created_at=g.created_at, status=GatewayStatus(g.status),
                   status_message=g.status_message, hostname=comp.hostname if comp else None,
                   ip_address=comp.ip_address if comp else None, instance_id=comp.instance_id if comp else None,
                   backend=conf.backend, region=g.region, default=g.project.default_gateway_id == g.id,
                   wildcard_domain=g.wildcard_domain)


def list_project_gateways(s: Session, project: ProjectModel) -> List[GatewayModel]:
    return list(s.execute(select(GatewayModel).where(GatewayModel.project_id == project.id)).scalars())


def get_gateway_by_name(s: Session, project: ProjectModel, name: str) -> Optional[GatewayModel]:
    return s.execute(select(GatewayModel).where(GatewayModel.project_id == project.id,
                                                GatewayModel.name == name)).scalar_one_or_none()


def get_plan(s: Session, project: ProjectModel, user: UserModel, spec: GatewaySpec) -> GatewayPlan:
    cur = get_gateway_by_name(s, project, spec.configuration.name) if spec.configuration.name else None
    return GatewayPlan(project_name=project.name, user=user.name, spec=spec,
                       current_resource=gateway_model_to_gateway(cur) if cur else None)


def create_gateway(s: Session, project: ProjectModel, conf: GatewayConfiguration) -> Gateway:
    if conf.backend not in BACKENDS_WITH_GATEWAY_SUPPORT:
        raise ServerClientError(f"Backend {conf.backend.value} does not support gateways")
    if not conf.public_ip and conf.backend not in BACKENDS_WITH_PRIVATE_GATEWAY_SUPPORT:
        raise ServerClientError(f"Backend {conf.backend.value} does not support gateways without a public IP")
    if conf.name is None:
        conf.name = generate_name()
    if get_gateway_by_name(s, project, conf.name) is not None:
        raise ResourceExistsError(f"Gateway {conf.name} exists")
    backend = s.execute(select(BackendModel).where(BackendModel.project_id == project.id,
                                                   BackendModel.type == conf.backend.value)).scalar_one_or_none()
    if backend is None:
        if conf.backend != BackendType.LOCAL:
            raise ServerClientError(f"Backend {conf.backend.value} is not configured")
        backend = BackendModel(id=uuid.uuid4(), project_id=project.id, type="local", config="{}", auth="{}")
        s.add(backend)
        s.flush()
    g = GatewayModel(id=uuid.uuid4(), name=conf.name, region=conf.region, project_id=project.id,
                     backend_id=backend.id, configuration=conf.model_dump_json(), status=GatewayStatus.SUBMITTED.value,
                     wildcard_domain=conf.domain, created_at=get_current_datetime(),
                     last_processed_at=get_current_datetime())
    s.add(g)
    s.flush()
    if conf.default or project.default_gateway_id is None:
        project.default_gateway_id = g.id
    scheduler.wake(scheduler.GATEWAYS)
    s.refresh(g)
    return gateway_model_to_gateway(g)


def _compute_configuration(g: GatewayModel):
    from dstack_amd.core.models.gateways import GatewayComputeConfiguration

    conf = GatewayConfiguration.model_validate_json(g.configuration) if g.configuration else None
    comp = g.gateway_compute
    if conf is None or comp is None:
        return None
    return GatewayComputeConfiguration(project_name=g.project.name, instance_name=g.name, backend=conf.backend,
                                       region=conf.region, public_ip=conf.public_ip,
                                       ssh_key_pub=comp.ssh_public_key or "", certificate=conf.certificate)


def terminate_gateway_compute(s: Session, g: GatewayModel) -> bool:
    """Terminate the gateway's VM through its backend (reference
    ``S/services/gateways/__init__.py:226-255``); ``False`` when the cloud call failed (the gateway
    row is kept so the user can retry the delete instead of leaking a billed VM)."""
    comp = g.gateway_compute
    if comp is None or not comp.active or comp.deleted:
        return True
    conf = _compute_configuration(g)
    if conf is None or conf.backend == BackendType.LOCAL:
        return True
    from dstack_amd.server.services import backends as backends_services

    last = None
    for attempt in range(3):
        try:
            compute = backends_services.get_project_backend(s, g.project, conf.backend)
            logger.info("Deleting gateway compute %s (%s) of %s", comp.instance_id, conf.backend.value, g.name)
            compute.terminate_gateway(comp.instance_id, conf, comp.backend_data)
            logger.info("Deleted gateway compute of %s", g.name)
            return True
        except Exception as e:  # noqa: BLE001
            last = e
            logger.warning("Deleting gateway compute of %s failed (attempt %d): %s", g.name, attempt + 1, e)
            import time

            time.sleep(0.2 * (attempt + 1))
    logger.error("Gateway %s kept: its compute %s could not be terminated: %s", g.name, comp.instance_id, last)
    return False


def delete_gateways(s: Session, project: ProjectModel, names: List[str]):
    gws = []
    for n in names:
        g = get_gateway_by_name(s, project, n)
        if g is None:
            raise ResourceNotExistsError(f"Gateway {n} not found")
        gws.append(g)
    failed = []
    for g in gws:
        if not terminate_gateway_compute(s, g):
            failed.append(g.name)
            continue
        if project.default_gateway_id == g.id:
            project.default_gateway_id = None
        if g.gateway_compute:
            _drop_tunnel(g)
            g.gateway_compute.active = False
            g.gateway_compute.deleted = True
        local = LocalGatewayProcess._instances.pop(f"{project.name}/{g.name}", None)
        if local is not None:
            local.stop()
        # runs keep their history without the gateway (the reference's ON DELETE SET NULL)
        s.query(RunModel).filter(RunModel.gateway_id == g.id).update({RunModel.gateway_id: None},
                                                                       synchronize_session="fetch")
        s.delete(g)
    if failed:
        s.commit()  # the gateways that were terminated stay deleted
        raise GatewayError(f"Failed to terminate the compute of gateway(s) {', '.join(failed)}; retry the delete")


def _drop_tunnel(g: GatewayModel):
    comp = g.gateway_compute
    data = json.loads(comp.backend_data or "{}")
    if data.get("api_url") or not comp.ip_address:
        return
    from dstack_amd.core.services.ssh.tunnel import SSHTarget, get_tunnel_pool

    try:
        get_tunnel_pool().close(SSHTarget(comp.ip_address, data.get("ssh_user", "ubuntu"), int(data.get("ssh_port", 22))))
    except Exception as e:  # noqa: BLE001
        logger.debug("closing gateway tunnel: %s", e)


def set_default_gateway(s: Session, project: ProjectModel, name: str):
    g = get_gateway_by_name(s, project, name)
    if g is None:
        raise ResourceNotExistsError()
    project.default_gateway_id = g.id


def set_wildcard_domain(s: Session, project: ProjectModel, name: str, domain: Optional[str]) -> Gateway:
    g = get_gateway_by_name(s, project, name)
    if g is None:
        raise ResourceNotExistsError()
    g.wildcard_domain = domain
    return gateway_model_to_gateway(g)


# ---------------------------------------------------------------------------------------------
# gateway API client
# ---------------------------------------------------------------------------------------------
def _gateway_url(g: GatewayModel) -> Optional[str]:
    comp = g.gateway_compute
    if comp is None:
        return None
    data = json.loads(comp.backend_data or "{}")
    if data.get("api_url"):
        return data["api_url"]  # local / trusted-LAN gateway
    # cloud gateway: the control API listens on the gateway's loopback; reach it over SSH
    from dstack_amd.core.services.ssh.tunnel import SSHTarget, get_tunnel_pool

    target = SSHTarget(comp.ip_address, data.get("ssh_user", "ubuntu"), int(data.get("ssh_port", 22)))
    local = get_tunnel_pool().forward(target, comp.ssh_private_key, int(data.get("control_port", 8000)))
    return f"http://127.0.0.1:{local}"


class LocalGatewayProcess:
    """A gateway for the ``local`` backend: ``dstack_amd.proxy.gateway.main`` on the server host
    (built-in data plane unless nginx is installed)."""

    _instances: dict = {}

    def __init__(self, name: str, state_dir: str, server_url: str):
        import subprocess
        import sys

        from dstack_amd.server.testing import free_port

        self.control_port, self.http_port = free_port(), free_port()
        self.proc = subprocess.Popen(
            [sys.executable, "-m", "dstack_amd.proxy.gateway.main", "--state-dir", state_dir, "--control-port",
             str(self.control_port), "--http-port", str(self.http_port), "--server-url", server_url,
             "--data-plane", "builtin"], stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
            start_new_session=True)
        for _ in range(300):
            try:
                if httpx.get(f"http://127.0.0.1:{self.control_port}/api/healthcheck", timeout=1).status_code == 200:
                    break
            except httpx.HTTPError:
                pass
            if self.proc.poll() is not None:
                raise GatewayError("local gateway exited during startup")
            import time

            time.sleep(0.1)
        LocalGatewayProcess._instances[name] = self

    def stop(self):
        if self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(10)
            except Exception:  # noqa: BLE001
                self.proc.kill()

    @classmethod
    def stop_all(cls):
        for gw in list(cls._instances.values()):
            gw.stop()
        cls._instances.clear()


def _call(g: GatewayModel, method: str, path: str, body: Optional[dict] = None) -> dict:
    url = _gateway_url(g)
    if url is None:
        raise GatewayError(f"gateway {g.name} is not provisioned")
    r = httpx.request(method, url + path, json=body, timeout=30)
    if r.status_code >= 400:
        raise GatewayError(f"gateway {g.name}: {r.status_code} {r.text}")
    return r.json() if r.content else {}


def gateway_register_service(s: Session, run: RunModel):
    g = s.get(GatewayModel, run.gateway_id)
    spec = RunSpec.model_validate_json(run.run_spec)
    conf = spec.configuration
    body = {"run_name": run.run_name, "domain": f"{run.run_name}.{g.wildcard_domain}", "https": conf.https,
            "auth": conf.auth, "client_max_body_size": 64 * 2**20,
            "options": {"openai": {"model": conf.model.model_dump()}} if conf.model else {}}
    _call(g, "POST", f"/api/registry/{run.project.name}/services/register", body)
    if conf.model is not None:
        _call(g, "POST", f"/api/registry/{run.project.name}/entrypoints/register",
              {"domain": f"gateway.{g.wildcard_domain}", "https": conf.https})


def gateway_unregister_service(s: Session, run: RunModel):
    g = s.get(GatewayModel, run.gateway_id) if run.gateway_id else None
    if g is None:
        return
    try:
        _call(g, "POST", f"/api/registry/{run.project.name}/services/{run.run_name}/unregister")
    except GatewayError as e:
        logger.info("unregister service: %s", e)


def gateway_register_replica(s: Session, run: RunModel, job: JobModel):
    g = s.get(GatewayModel, run.gateway_id)
    jpd = jobs_services.job_jpd(job)
    spec = RunSpec.model_validate_json(run.run_spec)
    jrd = jobs_services.job_jrd(job)
    port = spec.configuration.port.container_port
    if jrd is not None and jrd.ports:
        port = int(jrd.ports.get(port, jrd.ports.get(str(port), port)))
    direct = jpd.backend == BackendType.LOCAL or bool(json.loads(jpd.backend_data or "{}").get("direct"))
    body = {"job_id": str(job.id), "app_port": port, "ssh_host": f"{jpd.username}@{jpd.hostname}",
            "ssh_port": jpd.ssh_port or 22, "internal_ip": jpd.internal_ip or jpd.hostname, "direct": direct}
    try:
        _call(g, "POST", f"/api/registry/{run.project.name}/services/{run.run_name}/replicas/register", body)
    except GatewayError as e:
        logger.warning("register replica: %s", e)


def gateway_unregister_replica(s: Session, run: RunModel, job: JobModel):
    g = s.get(GatewayModel, run.gateway_id)
    if g is None:
        return
    try:
        _call(g, "POST", f"/api/registry/{run.project.name}/services/{run.run_name}/replicas/{job.id}/unregister")
    except GatewayError as e:
        logger.info("unregister replica: %s", e)


def gateway_stats(g: GatewayModel) -> dict:
    return _call(g, "GET", "/api/stats/collect")


# a cloud gateway VM boots and starts its app within minutes; one that cannot be reached for this
# long after its creation is marked FAILED (reference process_gateways: "Failed to connect")
GATEWAY_CONNECT_DEADLINE = 10 * 60


def connect_gateway(s: Session, g: GatewayModel) -> None:
    """PROVISIONING -> RUNNING once the gateway's control API answers (over the SSH tunnel for a
    cloud gateway), then its config (server URL, ACME) is pushed; FAILED after the deadline."""
    try:
        _call(g, "GET", "/api/healthcheck")
    except Exception as e:  # noqa: BLE001 - unreachable yet: retried on the next pass
        created = g.created_at.replace(tzinfo=None) if g.created_at else get_current_datetime()
        age = (get_current_datetime() - created).total_seconds()
        if age > GATEWAY_CONNECT_DEADLINE:
            g.status = GatewayStatus.FAILED.value
            g.status_message = f"Failed to connect to gateway: {e}"[:1000]
        return
    from dstack_amd.server import settings

    try:
        _call(g, "POST", "/api/config", {"server_url": settings.SERVER_URL})
    except Exception as e:  # noqa: BLE001 - configuration is re-pushed at server start
        logger.warning("gateway %s: configure failed: %s", g.name, e)
    g.status = GatewayStatus.RUNNING.value
    g.status_message = None


def provision_gateway(s: Session, g: GatewayModel):
    """SUBMITTED -> PROVISIONING (-> RUNNING in ``connect_gateway``).  ``local`` gateways run
    in-process on the server host and are RUNNING at once; cloud gateways need the backend's
    ``create_gateway`` (cloud API)."""
    conf = GatewayConfiguration.model_validate_json(g.configuration)
    if conf.backend == BackendType.LOCAL:
        from dstack_amd.server import settings

        private, public = generate_rsa_key_pair("dstack-gateway")
        try:
            proc = LocalGatewayProcess(f"{g.project.name}/{g.name}",
                                       str(settings.SERVER_DIR_PATH / "gateways" / g.project.name / g.name),
                                       settings.SERVER_URL)
        except GatewayError as e:
            g.status = GatewayStatus.FAILED.value
            g.status_message = str(e)
            return
        comp = GatewayComputeModel(id=uuid.uuid4(), instance_id="local", ip_address="127.0.0.1",
                                   hostname=f"127.0.0.1:{proc.http_port}", region="local", backend_id=g.backend_id,
                                   ssh_private_key=private, ssh_public_key=public,
                                   configuration=conf.model_dump_json(),
                                   backend_data=json.dumps({"api_url": f"http://127.0.0.1:{proc.control_port}",
                                                            "http_port": proc.http_port}))
        s.add(comp)
        s.flush()
        g.gateway_compute_id = comp.id
        g.status = GatewayStatus.RUNNING.value
        return
    from dstack_amd.server.services import backends as backends_services

    try:
        compute = backends_services.get_project_backend(s, g.project, conf.backend)
        from dstack_amd.core.models.gateways import GatewayComputeConfiguration

        private, public = generate_rsa_key_pair("dstack-gateway")
        gpd = compute.create_gateway(GatewayComputeConfiguration(
            project_name=g.project.name, instance_name=g.name, backend=conf.backend, region=conf.region,
            public_ip=conf.public_ip, ssh_key_pub=public, certificate=conf.certificate))
    except Exception as e:  # noqa: BLE001
        g.status = GatewayStatus.FAILED.value
        g.status_message = str(e)[:1000]
        return
    comp = GatewayComputeModel(id=uuid.uuid4(), instance_id=gpd.instance_id, ip_address=gpd.ip_address,
                               hostname=gpd.hostname, region=gpd.region, backend_id=g.backend_id,
                               ssh_private_key=private, ssh_public_key=public, backend_data=gpd.backend_data)
    s.add(comp)
    s.flush()
    g.gateway_compute_id = comp.id
    g.status = GatewayStatus.PROVISIONING.value


# ---------------------------------------------------------------------------------------------
# server start: reconnect, blue/green app update, configure (reference
# ``S/services/gateways/__init__.py:356-430``)
# ---------------------------------------------------------------------------------------------
UPDATE_COOLDOWN_S = 60


def _ssh_target(comp: GatewayComputeModel):
    from dstack_amd.core.services.ssh.tunnel import SSHTarget

    data = json.loads(comp.backend_data or "{}")
    return SSHTarget(comp.ip_address, data.get("ssh_user", "ubuntu"), int(data.get("ssh_port", 22)))


def update_gateway_app(comp: GatewayComputeModel, version: Optional[str] = None, url: Optional[str] = None) -> bool:
    """Push the server's ``update.sh`` and run the blue/green update to ``version`` on the gateway
    host over SSH; True when the new app reported healthy (else update.sh rolled back)."""
    from dstack_amd import __version__
    from dstack_amd.core.services.ssh.tunnel import get_tunnel_pool
    from dstack_amd.proxy.gateway import packaging

    version = version or __version__
    url = url or packaging.package_url(version)
    pool, target = get_tunnel_pool(), _ssh_target(comp)
    r = pool.run(target, comp.ssh_private_key, "mkdir -p dstack && cat > dstack/update.sh",
                 input=packaging.UPDATE_SH.encode(), timeout=60)
    if r.returncode != 0:
        raise GatewayError(f"pushing update.sh failed: {r.stderr.decode(errors='replace')[-300:]}")
    r = pool.run(target, comp.ssh_private_key, packaging.remote_update_command(url, version), timeout=600)
    out = r.stdout.decode(errors="replace")
    if "Update successfully completed" in out:
        logger.info("Gateway %s updated to %s", comp.ip_address, version)
        return True
    logger.warning("Gateway %s update to %s failed: %s", comp.ip_address, version, out[-500:])
    return False


def _recently_updated(comp: GatewayComputeModel) -> bool:
    from datetime import timedelta

    t = comp.app_updated_at
    if t is None:
        return False
    now = get_current_datetime()
    if t.tzinfo is None:
        now = now.replace(tzinfo=None)
    return t > now - timedelta(seconds=UPDATE_COOLDOWN_S)


def _restart_local_gateway(s: Session, g: GatewayModel) -> str:
    """A ``local`` gateway runs as a child of the server: after a server restart it is relaunched
    on its persisted state (registered services and replicas come back from state-v2.json)."""
    from dstack_amd.server import settings

    key = f"{g.project.name}/{g.name}"
    cur = LocalGatewayProcess._instances.get(key)
    if cur is not None and cur.proc.poll() is None:
        return "running"
    proc = LocalGatewayProcess(key, str(settings.SERVER_DIR_PATH / "gateways" / g.project.name / g.name),
                               settings.SERVER_URL)
    comp = g.gateway_compute
    data = json.loads(comp.backend_data or "{}")
    data.update(api_url=f"http://127.0.0.1:{proc.control_port}", http_port=proc.http_port)
    comp.backend_data = json.dumps(data)
    comp.hostname = f"127.0.0.1:{proc.http_port}"
    return "restarted"


def _init_one(gateway_id, skip_update: bool) -> str:
    from dstack_amd import __version__
    from dstack_amd.server import settings
    from dstack_amd.server.db import session_scope

    with session_scope() as s:
        g = s.get(GatewayModel, gateway_id)
        if g is None or g.gateway_compute is None:
            return "gone"
        if BackendType(g.backend.type) == BackendType.LOCAL:
            return _restart_local_gateway(s, g)
        comp = g.gateway_compute
        try:
            health = _call(g, "GET", "/api/healthcheck")
        except Exception as e:  # noqa: BLE001 - an unreachable gateway must not block the server start
            logger.warning("Failed to connect to gateway %s: %s", comp.ip_address, e)
            return "unreachable"
        state = "connected"
        if health.get("version") != __version__ and not skip_update:
            if _recently_updated(comp):
                logger.debug("Skipping gateway %s update: updated recently", comp.ip_address)
            else:
                try:
                    if update_gateway_app(comp):
                        comp.app_updated_at = get_current_datetime()
                        state = "updated"
                    else:
                        state = "update_failed"
                except Exception as e:  # noqa: BLE001
                    logger.warning("Failed to update gateway %s: %s", comp.ip_address, e)
                    state = "update_failed"
        try:
            _call(g, "POST", "/api/config", {"server_url": settings.SERVER_URL})
        except Exception as e:  # noqa: BLE001
            logger.warning("Failed to configure gateway %s: %r", comp.ip_address, e)
        return state


def init_gateways(skip_update: Optional[bool] = None) -> dict:
    """Run at server start (before the reconcilers): every active gateway is reconnected, its app
    is updated blue/green when it runs another version than the server, and it is re-configured
    with the server URL; local gateways are relaunched.  Gateways are handled concurrently and a
    failing one is only logged.  Returns ``{gateway name: state}``."""
    from concurrent.futures import ThreadPoolExecutor

    from dstack_amd.server import settings
    from dstack_amd.server.db import session_scope
    from dstack_amd.server.services.locking import db_advisory_lock

    if skip_update is None:
        skip_update = settings.SKIP_GATEWAY_UPDATE
    with session_scope() as s:
        rows = s.execute(select(GatewayModel.id, GatewayModel.name).join(
            GatewayComputeModel, GatewayModel.gateway_compute_id == GatewayComputeModel.id).where(
            GatewayComputeModel.active.is_(True), GatewayComputeModel.deleted.is_(False))).all()
    if not rows:
        return {}
    logger.info("Connecting to %d gateway(s)...", len(rows))
    out = {}
    with db_advisory_lock(None, "gateway_tunnels"), ThreadPoolExecutor(max_workers=min(8, len(rows))) as ex:
        futs = {name: ex.submit(_init_one, gid, skip_update) for gid, name in rows}
        for name, f in futs.items():
            try:
                out[name] = f.result()
            except Exception as e:  # noqa: BLE001
                logger.warning("gateway %s init failed: %s", name, e)
                out[name] = "error"
    return out
