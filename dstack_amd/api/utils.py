"""Profile and configuration loading for Python API users (reference ``src/dstack/api/utils.py``)."""

from __future__ import annotations

import os
from pathlib import Path
from typing import Optional, Tuple, Union

import yaml

from dstack_amd.core.errors import ConfigurationError
from dstack_amd.core.models.profiles import Profile, ProfilesConfig
from dstack_amd.core.services.configs import get_dstack_dir

PathLike = Union[str, os.PathLike]


def _profiles_file(directory: Path) -> Path:
    p = directory / "profiles.yml"
    return p if p.exists() else p.with_suffix(".yaml")


def _from_file(path: Path, name: Optional[str]) -> Optional[Profile]:
    if not path.exists():
        return None
    try:
        data = yaml.safe_load(path.read_text()) or {}
    except yaml.YAMLError as e:
        raise ConfigurationError(f"Invalid YAML in {path}: {e}") from e
    cfg = ProfilesConfig.model_validate({"profiles": [], **data})
    if name is None:
        return cfg.default()
    return next((p for p in cfg.profiles if p.name == name), None)


def load_profile(repo_dir: PathLike, profile_name: Optional[str]) -> Profile:
    """The named profile (or the one marked ``default``) from the repo's ``.dstack/profiles.yml``,
    else from the user's ``~/.dstack/profiles.yml``; with no profiles at all an empty ``default``
    profile. An unknown name is a ConfigurationError."""
    for directory in (Path(repo_dir) / ".dstack", get_dstack_dir()):
        p = _from_file(_profiles_file(directory), profile_name)
        if p is not None:
            return p
    if profile_name is None:
        return Profile(name="default")
    raise ConfigurationError(f"No such profile: {profile_name}")


def load_configuration(repo_dir: PathLike, work_dir: Optional[PathLike] = None,
                       configuration_file: Optional[PathLike] = None) -> Tuple[str, object]:
    """(path relative to the repo, parsed run configuration): ``configuration_file`` or the
    ``.dstack.yml``/``.dstack.yaml`` in ``work_dir`` (default: the repo root), which must lie inside
    the repo."""
    from dstack_amd.core.models.configurations import parse_run_configuration

    repo = Path(repo_dir).resolve()
    wd = (repo / work_dir).resolve() if work_dir else repo
    if configuration_file is None:
        cands = [wd / ".dstack.yml", wd / ".dstack.yaml"]
        path = next((c for c in cands if c.exists()), None)
        if path is None:
            raise ConfigurationError(f"No .dstack.yml in {wd}")
    else:
        path = (wd / configuration_file).resolve()
    try:
        rel = path.relative_to(repo)
    except ValueError:
        raise ConfigurationError(f"{path} is outside the repo {repo}") from None
    if not path.exists():
        raise ConfigurationError(f"Configuration file {path} does not exist")
    try:
        data = yaml.safe_load(path.read_text())
    except yaml.YAMLError as e:
        raise ConfigurationError(f"Invalid YAML in {path}: {e}") from e
    return str(rel), parse_run_configuration(data or {})
