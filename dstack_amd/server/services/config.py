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

from pathlib import Path
from typing import List, Optional

import yaml
from pydantic import Field
from sqlalchemy.orm import Session

from dstack_amd.core.models.common import CoreModel
from dstack_amd.server import settings
from dstack_amd.server.models import UserModel
from dstack_amd.server.services import backends as backends_services
from dstack_amd.server.services import encryption
from dstack_amd.server.services import permissions as permissions_services
from dstack_amd.server.services import projects as projects_services


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
        if self.config is None:
            return
        for pc in self.config.projects:
            project = projects_services.get_or_create_default_project(s, owner, pc.name)
            existing = {b.type for b in project.backends}
            for b in pc.backends:
                if b.get("type") in existing:
                    backends_services.update_backend(s, project, b)
                else:
                    backends_services.create_backend(s, project, b)

    def init_config(self, project_name: str):
        if self.path.exists():
            return
        self.path.parent.mkdir(parents=True, exist_ok=True)
        self.path.write_text(yaml.safe_dump({"projects": [{"name": project_name, "backends": []}]}))
