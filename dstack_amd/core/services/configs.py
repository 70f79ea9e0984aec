"""Client-side ``~/.dstack/config.yml`` (projects + initialised repos) — reference:
``core/services/configs/__init__.py:21-140``, ``core/models/config.py:8-24``.

Writes go through a file lock and an atomic rename so concurrent CLI invocations
(``dstack init`` in two shells) cannot corrupt the file.
"""

from __future__ import annotations

import os
import tempfile
from pathlib import Path
from typing import List, Optional

import filelock
import yaml
from pydantic import ValidationError

from dstack_amd.core.models.common import CoreModel


class ProjectConfig(CoreModel):
    name: str
    url: str
    token: str
    default: Optional[bool] = None


class RepoConfig(CoreModel):
    path: str
    repo_id: str
    repo_type: str
    ssh_key_path: str


class GlobalConfig(CoreModel):
    projects: List[ProjectConfig] = []
    repos: List[RepoConfig] = []


def get_dstack_dir() -> Path:
    return Path(os.environ.get("DSTACK_DIR", str(Path.home() / ".dstack")))


class ConfigManager:
    def __init__(self, dstack_dir: Optional[os.PathLike] = None):
        self.dstack_dir = Path(dstack_dir) if dstack_dir else get_dstack_dir()
        self.config_filepath = self.dstack_dir / "config.yml"
        self.load()

    @property
    def dstack_ssh_dir(self) -> Path:
        return self.dstack_dir / "ssh"

    @property
    def dstack_key_path(self) -> Path:
        return self.dstack_ssh_dir / "id_rsa"

    def load(self):
        try:
            with open(self.config_filepath) as f:
                self.config = GlobalConfig.model_validate(yaml.safe_load(f) or {})
        except (FileNotFoundError, ValidationError):
            self.config = GlobalConfig()

    def save(self):
        self.dstack_dir.mkdir(parents=True, exist_ok=True)
        fd, tmp = tempfile.mkstemp(dir=self.dstack_dir, prefix=".config.")
        with os.fdopen(fd, "w") as f:
            yaml.safe_dump(self.config.model_dump(mode="json", exclude_none=True), f, sort_keys=False)
        os.replace(tmp, self.config_filepath)

    def _locked(self):
        self.dstack_dir.mkdir(parents=True, exist_ok=True)
        return filelock.FileLock(str(self.config_filepath) + ".lock")

    # ---- projects -----------------------------------------------------------------------------
    def get_project_config(self, name: Optional[str] = None) -> Optional[ProjectConfig]:
        for p in self.config.projects:
            if (name is None and p.default) or p.name == name:
                return p
        if name is None and len(self.config.projects) == 1:
            return self.config.projects[0]
        return None

    def configure_project(self, name: str, url: str, token: str, default: bool = False):
        if default:
            for p in self.config.projects:
                p.default = False
        for p in self.config.projects:
            if p.name == name:
                p.url, p.token = url, token
                p.default = default or p.default
                return
        self.config.projects.append(ProjectConfig(name=name, url=url, token=token, default=default))
        if len(self.config.projects) == 1:
            self.config.projects[0].default = True

    def delete_project(self, name: str):
        self.config.projects = [p for p in self.config.projects if p.name != name]

    # ---- repos --------------------------------------------------------------------------------
    def save_repo_config(self, repo_path: os.PathLike, repo_id: str, repo_type: str, ssh_key_path: os.PathLike):
        with self._locked():
            self.load()
            repo_path, ssh_key_path = os.path.abspath(repo_path), os.path.abspath(ssh_key_path)
            for r in self.config.repos:
                if r.path == repo_path:
                    r.repo_id, r.repo_type, r.ssh_key_path = repo_id, repo_type, ssh_key_path
                    break
            else:
                self.config.repos.append(RepoConfig(path=repo_path, repo_id=repo_id, repo_type=repo_type,
                                                    ssh_key_path=ssh_key_path))
            self.save()

    def get_repo_config(self, repo_path: os.PathLike) -> Optional[RepoConfig]:
        repo_path = os.path.abspath(repo_path)
        return next((r for r in self.config.repos if r.path == repo_path), None)

    def ensure_ssh_key(self) -> Path:
        """The user's key pair for ``dstack attach`` / fleets (generated on first use)."""
        key = self.dstack_key_path
        if not key.exists():
            from dstack_amd.utils.common import generate_rsa_key_pair

            key.parent.mkdir(parents=True, exist_ok=True)
            private, public = generate_rsa_key_pair()
            fd = os.open(key, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
            with os.fdopen(fd, "w") as f:
                f.write(private)
            Path(str(key) + ".pub").write_text(public + "\n")
        return key
