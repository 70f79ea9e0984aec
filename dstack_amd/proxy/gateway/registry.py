"""Gateway registry: services, replicas and model entrypoints (reference:
``P/gateway/services/registry.py:31-354``, ``P/gateway/repo/repo.py``, state file
``~/dstack/state-v2.json``).

State is a plain JSON document written atomically after every change, so a gateway restart (or a
blue/green update) re-creates the nginx sites and the replica connections from it.

Replica reachability (MI355X on-prem first):
* ``direct``  — the gateway shares a trusted network with the hosts: the upstream is
  ``internal_ip:app_port`` (no per-replica SSH process);
* ``ssh``     — otherwise an ``ssh -N -L <unix socket>:localhost:<app_port>`` tunnel per replica
  through the pooled ControlMaster (``core/services/ssh/tunnel.py``), upstream ``unix:<socket>``.
"""

from __future__ import annotations

import json
import os
import tempfile
import threading
from dataclasses import asdict, dataclass, field
from pathlib import Path
from typing import Dict, List, Optional


@dataclass
class Replica:
    id: str
    app_port: int
    ssh_host: Optional[str] = None  # user@host
    ssh_port: int = 22
    ssh_proxy: Optional[str] = None  # user@host:port of a jump host
    internal_ip: Optional[str] = None
    mode: str = "direct"  # direct | ssh
    socket: Optional[str] = None  # unix socket of the ssh forward

    def upstream(self) -> str:
        if self.mode == "ssh" and self.socket:
            return f"unix:{self.socket}"
        return f"{self.internal_ip or '127.0.0.1'}:{self.app_port}"


@dataclass
class Service:
    project: str
    run_name: str
    domain: str
    https: bool = False
    auth: bool = True
    client_max_body_size: int = 64 * 2**20
    model: Optional[dict] = None  # {"name", "format", "prefix", "chat_template", "eos_token"}
    replicas: Dict[str, Replica] = field(default_factory=dict)

    @property
    def key(self) -> str:
        return f"{self.project}/{self.run_name}"


@dataclass
class Entrypoint:
    project: str
    domain: str
    https: bool = False


class RegistryError(ValueError):
    pass


class Registry:
    def __init__(self, state_path: Optional[Path] = None):
        self.state_path = state_path
        self._lock = threading.RLock()
        self.services: Dict[str, Service] = {}
        self.entrypoints: Dict[str, Entrypoint] = {}  # project -> entrypoint
        self.acme: dict = {}
        if state_path is not None and state_path.exists():
            self._load()

    # ---- persistence --------------------------------------------------------------------------
    def _load(self):
        d = json.loads(self.state_path.read_text())
        for s in d.get("services", []):
            reps = {r["id"]: Replica(**r) for r in s.pop("replicas", [])}
            svc = Service(**s)
            svc.replicas = reps
            self.services[svc.key] = svc
        for e in d.get("entrypoints", []):
            self.entrypoints[e["project"]] = Entrypoint(**e)
        self.acme = d.get("acme", {})

    def save(self):
        if self.state_path is None:
            return
        with self._lock:
            d = {"version": 2, "acme": self.acme,
                 "services": [dict(asdict(s), replicas=[asdict(r) for r in s.replicas.values()])
                              for s in self.services.values()],
                 "entrypoints": [asdict(e) for e in self.entrypoints.values()]}
        self.state_path.parent.mkdir(parents=True, exist_ok=True)
        fd, tmp = tempfile.mkstemp(dir=self.state_path.parent, prefix=".state.")
        with os.fdopen(fd, "w") as f:
            json.dump(d, f, indent=1)
        os.replace(tmp, self.state_path)

    # ---- services -----------------------------------------------------------------------------
    def register_service(self, project: str, run_name: str, domain: str, https: bool = False, auth: bool = True,
                         client_max_body_size: int = 64 * 2**20, model: Optional[dict] = None) -> Service:
        with self._lock:
            for s in self.services.values():
                if s.domain == domain and s.key != f"{project}/{run_name}":
                    raise RegistryError(f"domain {domain} is already used by {s.key}")
            key = f"{project}/{run_name}"
            if key in self.services:
                raise RegistryError(f"service {key} is already registered")
            svc = Service(project, run_name, domain, https, auth, client_max_body_size, model)
            self.services[key] = svc
        self.save()
        return svc

    def unregister_service(self, project: str, run_name: str) -> Service:
        with self._lock:
            svc = self.services.pop(f"{project}/{run_name}", None)
        if svc is None:
            raise RegistryError(f"service {project}/{run_name} is not registered")
        self.save()
        return svc

    def get_service(self, project: str, run_name: str) -> Optional[Service]:
        return self.services.get(f"{project}/{run_name}")

    def service_by_domain(self, host: str) -> Optional[Service]:
        host = host.split(":")[0].lower()
        for s in self.services.values():
            if s.domain.lower() == host:
                return s
        return None

    def add_replica(self, project: str, run_name: str, replica: Replica) -> Service:
        with self._lock:
            svc = self.services.get(f"{project}/{run_name}")
            if svc is None:
                raise RegistryError(f"service {project}/{run_name} is not registered")
            if replica.id in svc.replicas:
                raise RegistryError(f"replica {replica.id} of {project}/{run_name} is already registered")
            svc.replicas[replica.id] = replica
        self.save()
        return svc

    def remove_replica(self, project: str, run_name: str, replica_id: str) -> Optional[Replica]:
        with self._lock:
            svc = self.services.get(f"{project}/{run_name}")
            if svc is None:
                raise RegistryError(f"service {project}/{run_name} is not registered")
            rep = svc.replicas.pop(replica_id, None)
            if rep is None:
                raise RegistryError(f"replica {replica_id} of {project}/{run_name} is not registered")
        self.save()
        return rep

    # ---- model entrypoints --------------------------------------------------------------------
    def register_entrypoint(self, project: str, domain: str, https: bool = False) -> Entrypoint:
        with self._lock:
            ep = Entrypoint(project, domain, https)
            self.entrypoints[project] = ep
        self.save()
        return ep

    def entrypoint_by_domain(self, host: str) -> Optional[Entrypoint]:
        host = host.split(":")[0].lower()
        for e in self.entrypoints.values():
            if e.domain.lower() == host:
                return e
        return None

    def project_models(self, project: str) -> List[Service]:
        return [s for s in self.services.values() if s.project == project and s.model]
