"""Server ``config.yml`` (reference: ``S/services/config.py:509-676``):

.. code-block:: yaml

    projects:
      - name: main
        backends:
          - type: vultr
            creds: {type: api_key, api_key: ...}
    encryption:
      keys:
        - type: aes
          name: key1
          secret: <base64 32 bytes>
    default_permissions:
      allow_non_admins_create_projects: true
      allow_non_admins_manage_ssh_fleets: true
"""

from __future__ import annotations

import json
import logging
from pathlib import Path
from typing import List, Optional

import yaml
from pydantic import Field
from sqlalchemy.orm import Session

from dstack_amd.core.errors import ServerClientError
from dstack_amd.core.models.backend_configs import split_backend_config
from dstack_amd.core.models.common import CoreModel
from dstack_amd.server import settings
from dstack_amd.server.models import UserModel
from dstack_amd.server.services import backends as backends_services
from dstack_amd.server.services import encryption
from dstack_amd.server.services import permissions as permissions_services
from dstack_amd.server.services import projects as projects_services


logger = logging.getLogger(__name__)

# settings a backend records at creation (``prepare_backend_resources``: OCI's compartment and
# per-region subnets) that config.yml need not repeat
_PREPARED_KEYS = ("compartment_id", "subnet_ids")


def _unchanged(row, raw: dict) -> bool:
    """True when ``raw`` (a config.yml backend entry) would store exactly what ``row`` holds."""
    try:
        _, cfg, secrets = split_backend_config(raw)
    except (ValueError, TypeError):
        return False  # invalid: let create/update report it
    stored_cfg = json.loads(row.config or "{}")
    stored_secrets = json.loads(row.auth or "{}")
    for k in _PREPARED_KEYS:
        if k not in cfg:
            stored_cfg.pop(k, None)
    return stored_cfg == cfg and stored_secrets == secrets


class ProjectConfig(CoreModel):
    name: str
    backends: List[dict] = []


class EncryptionConfig(CoreModel):
    keys: List[dict] = []


DefaultPermissions = permissions_services.DefaultPermissions


class ServerConfig(CoreModel):
    projects: List[ProjectConfig] = Field(default_factory=list)
    encryption: Optional[EncryptionConfig] = None
    default_permissions: Optional[DefaultPermissions] = None


class ServerConfigManager:
    def __init__(self, path: Optional[Path] = None):
        self.path = Path(path or settings.SERVER_CONFIG_FILE_PATH)
        self.config: Optional[ServerConfig] = None

    def load_config(self) -> bool:
        if not self.path.exists():
            self.config = None
            permissions_services.set_default_permissions(None)
            return False
        data = yaml.safe_load(self.path.read_text()) or {}
        self.config = ServerConfig.model_validate(data)
        permissions_services.set_default_permissions(self.config.default_permissions)
        return True

    def apply_encryption(self):
        if self.config and self.config.encryption:
            encryption.configure_keys(self.config.encryption.keys)

    def apply_config(self, s: Session, owner: UserModel):
        """``config.yml`` is the source of truth for the backends of the projects it lists
        (reference ``services/config.py:550-616``): a listed backend is created, or updated when
        its settings or credentials changed (an unchanged one is skipped: no credential check
        against the cloud on every restart); a backend the project has but the file no longer
        lists is deleted -- unless it still owns live instances or volumes, which is logged and
        kept.  One backend that fails (invalid settings, rejected credentials) is logged and
        skipped: the server still starts with the others.  Projects the file does not list are
        left alone (their backends are managed through the API/UI)."""
        if self.config is None:
            return
        for pc in self.config.projects:
            self._apply_project_config(s, owner, pc)

    def _apply_project_config(self, s: Session, owner: UserModel, pc: ProjectConfig):
        project = projects_services.get_or_create_default_project(s, owner, pc.name)
        listed = set()
        for raw in pc.backends:
            try:
                btype = backends_services.configurable_type(raw)
            except ServerClientError as e:
                logger.warning("project %s: backend %r skipped: %s", pc.name, raw.get("type"), e)
                continue
            listed.add(btype.value)
            row = next((b for b in project.backends if b.type == btype.value), None)
            try:
                if row is not None and _unchanged(row, raw):
                    continue
                # (both validate settings and credentials before they write anything, so a failure
                # leaves this backend's row as it was)
                if row is None:
                    backends_services.create_backend(s, project, raw)
                else:
                    backends_services.update_backend(s, project, raw)
                logger.info("project %s: backend %s %s from %s", pc.name, btype.value,
                            "created" if row is None else "updated", self.path)
            except Exception as e:  # noqa: BLE001 - one bad backend must not stop the server
                logger.warning("project %s: failed to configure backend %s: %s", pc.name, btype.value, e)
        s.expire(project, ["backends"])
        for b in list(project.backends):
            if b.type in listed:
                continue
            try:
                backends_services.delete_backends(s, project, [b.type])  # (checks before it deletes)
                logger.info("project %s: backend %s deleted (no longer in %s)", pc.name, b.type, self.path)
            except ServerClientError as e:
                logger.warning("project %s: backend %s is no longer in %s but was kept: %s", pc.name, b.type,
                               self.path, e)

    def init_config(self, project_name: str):
        if self.path.exists():
            return
        self.path.parent.mkdir(parents=True, exist_ok=True)
        self.path.write_text(yaml.safe_dump({"projects": [{"name": project_name, "backends": []}]}))
