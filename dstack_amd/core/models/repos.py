"""Repos: what code a run gets (reference: ``C/models/repos/*``).

* ``RemoteRepo`` — a git checkout with a remote; the run clones ``repo_hash`` and applies the local
  uncommitted diff (``git diff`` incl. untracked files) on top.  Implemented with the ``git`` CLI.
* ``LocalRepo``  — a directory shipped as a tarball (respecting ``.gitignore``/``.dstackignore``).
* ``VirtualRepo`` — in-memory files (programmatic API).
"""

from __future__ import annotations

import fnmatch
import hashlib
import io
import os
import re
import urllib.parse
import subprocess
import tarfile
from abc import ABC, abstractmethod
from enum import Enum
from typing import BinaryIO, Dict, List, Literal, Optional, Union

from pydantic import Field
from typing_extensions import Annotated

from dstack_amd.core.errors import DstackError
from dstack_amd.core.models.common import CoreModel


class RepoType(str, Enum):
    REMOTE = "remote"
    LOCAL = "local"
    VIRTUAL = "virtual"


class RepoProtocol(str, Enum):
    SSH = "ssh"
    HTTPS = "https"


class RepoError(DstackError):
    pass


class RemoteRepoCreds(CoreModel):
    protocol: RepoProtocol = RepoProtocol.HTTPS
    clone_url: str
    private_key: Optional[str] = None
    oauth_token: Optional[str] = None


class RemoteRepoInfo(CoreModel):
    repo_type: Literal["remote"] = "remote"
    repo_name: str
    repo_host_name: str = ""
    repo_port: Optional[int] = None
    repo_user_name: str = ""


class RemoteRunRepoData(RemoteRepoInfo):
    repo_branch: Optional[str] = None
    repo_hash: Optional[str] = None
    repo_diff: Optional[str] = Field(None, exclude=True)
    repo_config_name: Optional[str] = None
    repo_config_email: Optional[str] = None


class LocalRepoInfo(CoreModel):
    repo_type: Literal["local"] = "local"
    repo_dir: str


class LocalRunRepoData(LocalRepoInfo):
    pass


class VirtualRepoInfo(CoreModel):
    repo_type: Literal["virtual"] = "virtual"


class VirtualRunRepoData(VirtualRepoInfo):
    pass


AnyRepoInfo = Annotated[Union[RemoteRepoInfo, LocalRepoInfo, VirtualRepoInfo], Field(discriminator="repo_type")]
AnyRunRepoData = Annotated[
    Union[RemoteRunRepoData, LocalRunRepoData, VirtualRunRepoData], Field(discriminator="repo_type")
]


class RepoHead(CoreModel):
    repo_id: str
    repo_info: AnyRepoInfo


class RepoHeadWithCreds(RepoHead):
    repo_creds: Optional[RemoteRepoCreds] = None


DEFAULT_VIRTUAL_REPO_ID = "none"


class Repo(ABC):
    repo_id: str
    repo_dir: Optional[str]
    run_repo_data: object

    @abstractmethod
    def write_code_file(self, fp: BinaryIO) -> str:
        """Write the code blob (diff or tar) and return its sha256."""

    @abstractmethod
    def get_repo_info(self):
        pass


class VirtualRepo(Repo):
    def __init__(self, repo_id: str = DEFAULT_VIRTUAL_REPO_ID, files: Optional[Dict[str, bytes]] = None):
        self.repo_id = repo_id
        self.repo_dir = None
        self.files: Dict[str, bytes] = dict(files or {})
        self.run_repo_data = VirtualRunRepoData()

    def add_file(self, path: str, content: Union[str, bytes]):
        if os.path.isabs(path) or ".." in path.split("/"):
            raise RepoError(f"invalid virtual repo path: {path}")
        self.files[path] = content.encode() if isinstance(content, str) else content

    def write_code_file(self, fp: BinaryIO) -> str:
        return _write_tar(fp, sorted(self.files.items()))

    def get_repo_info(self):
        return VirtualRepoInfo()


_DEFAULT_IGNORE = [".git", "__pycache__", "*.pyc", ".venv", "node_modules", ".dstack"]


def _load_ignore(repo_dir: str) -> List[str]:
    pats = list(_DEFAULT_IGNORE)
    for name in (".gitignore", ".dstackignore"):
        p = os.path.join(repo_dir, name)
        if os.path.exists(p):
            for line in open(p, encoding="utf-8", errors="ignore"):
                line = line.strip()
                if line and not line.startswith("#") and not line.startswith("!"):
                    pats.append(line.rstrip("/"))
    return pats


def _ignored(rel: str, pats: List[str]) -> bool:
    parts = rel.split("/")
    for pat in pats:
        anchored = pat.startswith("/")
        p = pat.lstrip("/")
        if "/" in p or anchored:
            if fnmatch.fnmatch(rel, p) or rel.startswith(p + "/"):
                return True
        elif any(fnmatch.fnmatch(part, p) for part in parts):
            return True
    return False


def _write_tar(fp: BinaryIO, items) -> str:
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w:gz", format=tarfile.PAX_FORMAT) as tar:
        for path, data in items:
            info = tarfile.TarInfo(path)
            info.size = len(data)
            info.mode = 0o644
            info.mtime = 0
            tar.addfile(info, io.BytesIO(data))
    blob = buf.getvalue()
    fp.write(blob)
    return hashlib.sha256(blob).hexdigest()


class LocalRepo(Repo):
    def __init__(self, repo_dir: str, repo_id: Optional[str] = None):
        self.repo_dir = os.path.abspath(repo_dir)
        self.repo_id = repo_id or hashlib.sha1(self.repo_dir.encode()).hexdigest()[:16]
        self.run_repo_data = LocalRunRepoData(repo_dir=self.repo_dir)

    def files(self):
        pats = _load_ignore(self.repo_dir)
        for root, dirs, files in os.walk(self.repo_dir):
            rel_root = os.path.relpath(root, self.repo_dir)
            rel_root = "" if rel_root == "." else rel_root
            dirs[:] = sorted(d for d in dirs if not _ignored(os.path.join(rel_root, d).lstrip("/"), pats))
            for f in sorted(files):
                rel = os.path.join(rel_root, f).lstrip("/")
                if not _ignored(rel, pats):
                    yield rel

    def write_code_file(self, fp: BinaryIO) -> str:
        items = []
        for rel in self.files():
            with open(os.path.join(self.repo_dir, rel), "rb") as f:
                items.append((rel, f.read()))
        return _write_tar(fp, items)

    def get_repo_info(self):
        return LocalRepoInfo(repo_dir=self.repo_dir)


_GIT_URL_RE = re.compile(r"^(?:(?P<scheme>[a-z+]+)://)?(?:(?P<user>[^@/]+)@)?(?P<host>[^:/]+)(?::(?P<port>\d+))?[:/](?P<path>.+?)(?:\.git)?/?$")


def parse_git_url(url: str) -> Dict[str, Optional[str]]:
    m = _GIT_URL_RE.match(url.strip())
    if not m:
        raise RepoError(f"cannot parse git url: {url}")
    return m.groupdict()


class GitRepoURL:
    """A git remote as the run will clone it (reference ``core/models/repos/remote.py``
    ``GitRepoURL``).  ``ssh://`` URLs and scp-style ``user@host:path`` locations name an SSH host
    that ``~/.ssh/config`` may alias (HostName / User / Port); an https URL keeps its host, and the
    SSH form of it takes the user and port the config gives that host."""

    def __init__(self, scheme: str, host: str, path: str, user: Optional[str] = None, port: Optional[int] = None,
                 ssh_user: Optional[str] = None, ssh_port: Optional[int] = None):
        self.scheme, self.host, self.path = scheme, host, path.lstrip("/")
        self.user, self.port = user, port
        self.ssh_user, self.ssh_port = ssh_user, ssh_port

    @classmethod
    def parse(cls, url: str, get_ssh_config=None) -> "GitRepoURL":
        from dstack_amd.utils.ssh import get_ssh_config as _default

        lookup = get_ssh_config or _default
        url = url.strip()
        if "://" in url:
            u = urllib.parse.urlsplit(url)
            if u.scheme not in ("https", "http", "ssh", "git+ssh") or not u.hostname or not u.path.strip("/"):
                raise RepoError(f"unsupported git url: {url}")
            if u.scheme in ("https", "http"):
                cfg = lookup(u.hostname) or {}
                return cls(u.scheme, u.hostname, u.path, port=u.port, ssh_user=cfg.get("user"),
                           ssh_port=int(cfg["port"]) if cfg.get("port") else None)
            cfg = lookup(u.hostname) or {}
            port = u.port or (int(cfg["port"]) if cfg.get("port") else None)
            return cls("ssh", cfg.get("hostname") or u.hostname, u.path, user=u.username or cfg.get("user"),
                       ssh_user=u.username or cfg.get("user"), ssh_port=port)
        m = re.match(r"^(?:(?P<user>[^@/:]+)@)?(?P<host>[^:/]+):(?P<path>[^/].*)$", url)
        if m is None:
            raise RepoError(f"cannot parse git url: {url}")
        cfg = lookup(m.group("host")) or {}
        user = m.group("user") or cfg.get("user")
        port = int(cfg["port"]) if cfg.get("port") else None
        return cls("ssh", cfg.get("hostname") or m.group("host"), m.group("path"), user=user, ssh_user=user,
                   ssh_port=port)

    def as_https(self, oauth_token: Optional[str] = None) -> str:
        auth = f"anything:{oauth_token}@" if oauth_token else ""
        port = f":{self.port}" if self.port and self.scheme in ("https", "http") else ""
        return f"https://{auth}{self.host}{port}/{self.path}"

    def as_ssh(self) -> str:
        user = self.ssh_user or "git"
        port = f":{self.ssh_port}" if self.ssh_port else ""
        return f"ssh://{user}@{self.host}{port}/{self.path}"


def _git(repo_dir: str, *args: str) -> str:
    r = subprocess.run(["git", "-C", repo_dir, *args], capture_output=True, text=True)
    if r.returncode != 0:
        raise RepoError(f"git {' '.join(args)} failed: {r.stderr.strip()}")
    return r.stdout


class RemoteRepo(Repo):
    """A local git checkout whose ``origin`` is reachable from the run."""

    def __init__(self, repo_dir: str, repo_url: Optional[str] = None, repo_id: Optional[str] = None):
        self.repo_dir = os.path.abspath(repo_dir)
        url = repo_url or _git(self.repo_dir, "config", "--get", "remote.origin.url").strip()
        self.repo_url = url
        parts = parse_git_url(url)
        host, path = parts["host"] or "", parts["path"] or ""
        self.repo_id = repo_id or hashlib.sha1(f"{host}/{path}".encode()).hexdigest()[:16]
        try:
            branch = _git(self.repo_dir, "rev-parse", "--abbrev-ref", "HEAD").strip()
        except RepoError:
            branch = None
        try:
            head = _git(self.repo_dir, "rev-parse", "HEAD").strip()
        except RepoError:
            head = None
        try:  # the host the run actually clones from (an ~/.ssh/config alias resolved)
            g = GitRepoURL.parse(url)
            r_host, r_user = g.host, g.ssh_user or parts["user"] or ""
            r_port = g.ssh_port if g.scheme == "ssh" else g.port
        except RepoError:
            r_host, r_user, r_port = host, parts["user"] or "", int(parts["port"]) if parts["port"] else None
        self.run_repo_data = RemoteRunRepoData(
            repo_name=path, repo_host_name=r_host, repo_port=r_port,
            repo_user_name=r_user, repo_branch=branch, repo_hash=head,
        )

    def diff(self) -> str:
        """Tracked changes vs HEAD plus untracked files (as /dev/null diffs)."""
        out = _git(self.repo_dir, "diff", "--binary", "HEAD")
        untracked = _git(self.repo_dir, "ls-files", "--others", "--exclude-standard").split("\n")
        for f in filter(None, untracked):
            r = subprocess.run(["git", "-C", self.repo_dir, "diff", "--binary", "--no-index", "/dev/null", f],
                               capture_output=True, text=True)
            out += r.stdout
        return out

    def write_code_file(self, fp: BinaryIO) -> str:
        data = self.diff().encode()
        fp.write(data)
        return hashlib.sha256(data).hexdigest()

    def get_repo_info(self):
        d = self.run_repo_data
        return RemoteRepoInfo(repo_name=d.repo_name, repo_host_name=d.repo_host_name, repo_port=d.repo_port,
                              repo_user_name=d.repo_user_name)


def code_hash(data: bytes) -> str:
    return hashlib.sha256(data).hexdigest()
