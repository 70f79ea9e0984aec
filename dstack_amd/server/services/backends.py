"""Backend registry, configurators and offer fan-out (reference:
``S/services/backends/__init__.py:36-451``, ``S/services/backends/configurators/*``).

A project's backends are rows of ``backends`` (type + JSON config + encrypted auth).  The ``local``
backend is implicit (enabled by ``DSTACK_LOCAL_BACKEND_ENABLED``); the ``remote`` backend (SSH
fleets) needs no configuration.  Cloud backends are configured with credentials; their offers
come from the built-in catalog (``core/backends/catalog.py``) or the cloud's live API, and they
provision through ``core/backends/clouds`` (REST clients, no vendor SDKs).
"""

from __future__ import annotations

import concurrent.futures as cf
import json
import threading
import time
import uuid
from typing import Dict, List, Optional, Tuple

from sqlalchemy import select
from sqlalchemy.orm import Session

from dstack_amd.core.backends.base import Compute
from dstack_amd.core.errors import BackendNotAvailable, ResourceExistsError, ResourceNotExistsError, ServerClientError
from dstack_amd.core.models.backend_configs import split_backend_config
from dstack_amd.core.models.backends import BackendType
from dstack_amd.core.models.instances import InstanceAvailability, InstanceOfferWithAvailability
from dstack_amd.core.models.runs import Requirements
from dstack_amd.server import settings
from dstack_amd.server.models import BackendModel, ProjectModel


def _make_compute(backend_type: BackendType, config: dict, auth: dict) -> Compute:
    if backend_type == BackendType.LOCAL:
        from dstack_amd.core.backends.local import LocalCompute

        return LocalCompute()
    if backend_type == BackendType.REMOTE:
        from dstack_amd.core.backends.remote import RemoteCompute

        return RemoteCompute()
    from dstack_amd.core.backends.clouds import compute_class

    cls = compute_class(backend_type)
    if backend_type == BackendType.KUBERNETES and auth.get("kubeconfig") and not config.get("kubeconfig"):
        config = {**config, "kubeconfig": auth["kubeconfig"]}  # stored with the secrets
    if cls is not None:
        return cls(config, auth)
    from dstack_amd.core.backends.catalog import CatalogCompute

    return CatalogCompute(backend_type, config, auth)


CONFIGURABLE_BACKENDS = [b for b in BackendType if b not in (BackendType.LOCAL, BackendType.REMOTE)]

_cache: Dict[Tuple[uuid.UUID, str, str], Compute] = {}
_cache_lock = threading.Lock()


def list_backend_types() -> List[str]:
    return [b.value for b in BackendType]


def get_project_backends(s: Session, project: ProjectModel) -> List[Tuple[BackendType, Compute]]:
    out: List[Tuple[BackendType, Compute]] = []
    rows = list(s.execute(select(BackendModel).where(BackendModel.project_id == project.id)).scalars())
    for row in rows:
        key = (project.id, row.type, row.config + "|" + (row.auth or ""))
        with _cache_lock:
            comp = _cache.get(key)
            if comp is None:
                comp = _make_compute(BackendType(row.type), json.loads(row.config or "{}"), json.loads(row.auth or "{}"))
                _cache[key] = comp
        out.append((BackendType(row.type), comp))
    if settings.LOCAL_BACKEND_ENABLED and not any(t == BackendType.LOCAL for t, _ in out):
        out.append((BackendType.LOCAL, get_local_compute()))
    return out


_local: Optional[Compute] = None
_remote: Optional[Compute] = None


def get_local_compute() -> Compute:
    global _local
    if _local is None:
        from dstack_amd.core.backends.local import LocalCompute

        _local = LocalCompute()
    return _local


def get_remote_compute() -> Compute:
    global _remote
    if _remote is None:
        from dstack_amd.core.backends.remote import RemoteCompute

        _remote = RemoteCompute()
    return _remote


def get_project_backend(s: Session, project: ProjectModel, backend_type: BackendType) -> Compute:
    if backend_type == BackendType.REMOTE:
        return get_remote_compute()
    for t, c in get_project_backends(s, project):
        if t == backend_type:
            return c
    raise BackendNotAvailable(f"Backend {backend_type.value} is not configured for project {project.name}")


def create_backend(s: Session, project: ProjectModel, config: dict) -> BackendModel:
    """Validate ``config`` against the backend's model (``core/models/backend_configs.py``) and
    store it: plain settings in ``config``, credentials in the encrypted ``auth`` column."""
    btype = configurable_type(config)
    existing = s.execute(select(BackendModel).where(BackendModel.project_id == project.id,
                                                    BackendModel.type == btype.value)).scalar_one_or_none()
    if existing is not None:
        raise ResourceExistsError(f"Backend {btype.value} exists")
    _, cfg, secrets = split_backend_config(config)
    _check_default_creds(secrets)
    validate_credentials(btype, cfg, secrets)
    cfg = prepare_backend_resources(btype, cfg, secrets)
    row = BackendModel(id=uuid.uuid4(), project_id=project.id, type=btype.value, config=json.dumps(cfg),
                       auth=json.dumps(secrets))
    s.add(row)
    s.flush()
    return row


def update_backend(s: Session, project: ProjectModel, config: dict) -> BackendModel:
    """Replace a backend's settings; credentials omitted from ``config`` keep their stored value."""
    btype = configurable_type(config)
    row = s.execute(select(BackendModel).where(BackendModel.project_id == project.id,
                                               BackendModel.type == btype.value)).scalar_one_or_none()
    if row is None:
        raise ResourceNotExistsError(f"Backend {btype.value} not found")
    merged = dict(config)
    old_secrets = json.loads(row.auth or "{}")
    if merged.get("creds") is None and btype != BackendType.KUBERNETES and old_secrets:
        merged["creds"] = old_secrets
    if btype == BackendType.KUBERNETES and merged.get("kubeconfig") is None and old_secrets.get("kubeconfig"):
        merged["kubeconfig"] = old_secrets["kubeconfig"]
    _, cfg, secrets = split_backend_config(merged)
    _check_default_creds(secrets)
    validate_credentials(btype, cfg, secrets)
    old_cfg = json.loads(row.config or "{}")
    for k in ("compartment_id", "subnet_ids"):  # keep what was bootstrapped unless overridden
        if k in old_cfg and k not in cfg and btype == BackendType.OCI:
            cfg[k] = old_cfg[k]
    cfg = prepare_backend_resources(btype, cfg, secrets)
    row.config = json.dumps(cfg)
    row.auth = json.dumps(secrets)
    return row


def _check_default_creds(secrets: dict) -> None:
    """``DSTACK_DEFAULT_CREDS_DISABLED``: ambient credentials (instance role, environment, metadata
    server) of the machine running the server may not be used by a project's backend."""
    from dstack_amd.server import settings

    if settings.DEFAULT_CREDS_DISABLED and secrets.get("type") == "default":
        raise ServerClientError("Default credentials are forbidden by dstack settings")


def validate_credentials(btype: BackendType, cfg: dict, secrets: dict) -> None:
    """Reference configurators' credential check: one authenticated call to the cloud.  Rejected
    credentials fail the request (``InvalidCredentialsError``, HTTP 400); an unreachable API (an
    air-gapped server, a network blip) does not -- the backend is stored and plans from the
    offline catalog until the cloud answers.  ``DSTACK_SKIP_BACKEND_VALIDATION=1`` skips it."""
    import logging
    import os

    import httpx

    from dstack_amd.core.errors import BackendAuthError, InvalidCredentialsError

    if os.getenv("DSTACK_SKIP_BACKEND_VALIDATION") == "1":
        return
    try:
        from dstack_amd.core.backends.clouds import compute_class

        cls = compute_class(btype)
        if cls is None:
            return
        if btype == BackendType.KUBERNETES and secrets.get("kubeconfig") and not cfg.get("kubeconfig"):
            cfg = {**cfg, "kubeconfig": secrets["kubeconfig"]}
        # a short timeout: an air-gapped server must not hold the request for the client's 60 s
        comp = cls(cfg, secrets, httpx.Client(timeout=float(os.getenv("DSTACK_BACKEND_VALIDATION_TIMEOUT", "15"))))
        check = getattr(comp, "check_credentials", None)
        if check is not None:
            check()
    except BackendAuthError as e:
        raise InvalidCredentialsError(f"Invalid {btype.value} credentials: {e}") from None
    except ServerClientError:
        raise  # a configuration the cloud refuses for another reason (e.g. unsubscribed regions)
    except (httpx.TransportError, OSError) as e:
        logging.getLogger(__name__).warning("%s credentials not verified (API unreachable: %s)", btype.value, e)
    except Exception as e:  # noqa: BLE001 -- e.g. a malformed key the signer cannot load
        raise InvalidCredentialsError(f"Invalid {btype.value} credentials: {e}") from None


def prepare_backend_resources(btype: BackendType, cfg: dict, secrets: dict) -> dict:
    """Cloud-side resources a backend needs before its first launch, created at backend creation
    and recorded in its stored config (OCI: compartment, VCN, subnet, gateway, routes, security
    rules).  Skipped with ``DSTACK_SKIP_BACKEND_VALIDATION=1`` (then created lazily at launch); an
    unreachable API is not an error either -- the launch path creates them idempotently."""
    import logging
    import os

    import httpx

    if os.getenv("DSTACK_SKIP_BACKEND_VALIDATION") == "1":
        return cfg
    from dstack_amd.core.backends.clouds import compute_class

    cls = compute_class(btype)
    if cls is None or not hasattr(cls, "prepare_config"):
        return cfg
    comp = cls(dict(cfg), secrets, httpx.Client(timeout=30.0))
    try:
        return {**cfg, **comp.prepare_config()}
    except (httpx.TransportError, OSError) as e:
        logging.getLogger(__name__).warning("%s resources not prepared (API unreachable: %s)", btype.value, e)
        return cfg


def configurable_type(config: dict) -> BackendType:
    try:
        btype = BackendType(config.get("type"))
    except ValueError:
        raise ServerClientError(f"Unknown backend type {config.get('type')!r}; one of: "
                                f"{', '.join(b.value for b in CONFIGURABLE_BACKENDS)}") from None
    if btype in (BackendType.LOCAL, BackendType.REMOTE):
        raise ServerClientError(f"{btype.value} backend needs no configuration")
    return btype


def delete_backends(s: Session, project: ProjectModel, names: List[str]):
    """Drop backend configurations, refused while any of them still owns live instances or
    volumes (their cloud resources could no longer be terminated or deleted)."""
    from dstack_amd.core.models.instances import InstanceStatus
    from dstack_amd.server.models import InstanceModel, VolumeModel

    busy = s.execute(select(InstanceModel.backend).where(
        InstanceModel.project_id == project.id, InstanceModel.backend.in_(names),
        InstanceModel.deleted == False,  # noqa: E712
        InstanceModel.status != InstanceStatus.TERMINATED.value)).scalars().first()
    if busy is not None:
        raise ServerClientError(f"Backend {busy} has active instances. Terminate them before deleting the backend.")
    for v in s.execute(select(VolumeModel).where(VolumeModel.project_id == project.id,
                                                 VolumeModel.deleted == False)).scalars():  # noqa: E712
        if json.loads(v.configuration or "{}").get("backend") in names:
            raise ServerClientError(f"Backend {json.loads(v.configuration)['backend']} has active volumes. "
                                    "Delete them before deleting the backend.")
    for n in names:
        row = s.execute(select(BackendModel).where(BackendModel.project_id == project.id,
                                                   BackendModel.type == n)).scalar_one_or_none()
        if row is not None:
            s.delete(row)


def backend_config_values(body: dict) -> dict:
    """Form choices for a backend: with ``creds`` given they are checked against the cloud first
    (rejected -> ``InvalidCredentialsError``, HTTP 400 ``invalid_credentials``), as the reference's
    configurators do before offering regions."""
    from dstack_amd.core.backends.catalog import offline_rows

    btype = configurable_type(body)
    if body.get("creds") is not None:
        try:
            _, cfg, secrets = split_backend_config(body)
        except ValueError:  # a form still being filled in: settings incomplete, creds checkable
            cfg = {k: v for k, v in body.items() if k not in ("type", "creds")}
            secrets = dict(body["creds"])
        _check_default_creds(secrets)
        validate_credentials(btype, cfg, secrets)
    regions = sorted({r.location for r in offline_rows(btype)})
    wanted = body.get("regions") or body.get("locations")
    selected = [r for r in regions if not wanted or r in wanted]
    return {"type": btype.value, "default_creds": btype in (BackendType.AWS, BackendType.AZURE, BackendType.GCP,
                                                             BackendType.OCI),
            "regions": {"selected": selected, "values": [{"value": r, "label": r} for r in regions]}}


def backend_config_info(s: Session, project: ProjectModel, name: str) -> dict:
    row = s.execute(select(BackendModel).where(BackendModel.project_id == project.id,
                                               BackendModel.type == name)).scalar_one_or_none()
    if row is None:
        raise ResourceNotExistsError()
    return {"type": row.type, **json.loads(row.config or "{}")}


def get_instance_offers(
    backends: List[Tuple[BackendType, Compute]], requirements: Requirements, exclude_not_available: bool = False,
) -> List[Tuple[Compute, InstanceOfferWithAvailability]]:
    """Query every backend concurrently, merge by price; unavailable offers last
    (``get_instance_offers`` ``S/services/backends/__init__.py:417-451``)."""
    results: List[Tuple[Compute, InstanceOfferWithAvailability]] = []
    if not backends:
        return results
    with cf.ThreadPoolExecutor(max_workers=min(8, len(backends))) as ex:
        futs = {ex.submit(c.get_offers_cached, requirements): c for _, c in backends}
        for fut in cf.as_completed(futs):
            comp = futs[fut]
            try:
                offers = fut.result()
            except Exception:  # noqa: BLE001 - a broken backend must not break planning
                continue
            results.extend((comp, o) for o in offers)
    if exclude_not_available:
        results = [r for r in results if r[1].availability.is_available()]
    results.sort(key=lambda r: (not r[1].availability.is_available(), r[1].price))
    return results
