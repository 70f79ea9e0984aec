"""Docker registry introspection (reference: ``S/services/docker.py:74-101``, python-dxf; cached
80 s in ``S/services/jobs/configurators/base.py:282-289``).

Reads an image's config (``User``, ``Entrypoint``, ``Cmd``, ``Env``) through the registry HTTP API
v2: bearer-token challenge (Docker Hub, GHCR, NGC, ECR-compatible), manifest list / OCI index ->
``linux/amd64`` manifest -> config blob.  Used when a configuration gives an ``image`` but no
``commands`` (run the image's own entrypoint) and to resolve the container user.
"""

from __future__ import annotations

import json
import threading
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import httpx
from pydantic import BaseModel, ConfigDict, Field, field_validator

from dstack_amd.core.errors import DockerRegistryError
from dstack_amd.server.utils.common import join_byte_stream_checked

MANIFEST_TYPES = ", ".join([
    "application/vnd.docker.distribution.manifest.list.v2+json",
    "application/vnd.oci.image.index.v1+json",
    "application/vnd.docker.distribution.manifest.v2+json",
    "application/vnd.oci.image.manifest.v1+json",
])
CACHE_TTL = 80.0


@dataclass
class ImageRef:
    registry: str
    repository: str
    reference: str  # tag or digest


@dataclass
class ImageConfig:
    user: Optional[str]
    entrypoint: Optional[List[str]]
    cmd: Optional[List[str]]
    env: List[str]


def parse_image_name(image: str) -> ImageRef:
    """``ubuntu`` -> docker.io/library/ubuntu:latest; ``ghcr.io/o/r:t``; ``reg:5000/r@sha256:..``"""
    name, digest = (image.split("@", 1) + [None])[:2]
    first, _, rest = name.partition("/")
    if rest and ("." in first or ":" in first or first == "localhost"):
        registry, path = first, rest
    else:
        registry, path = "registry-1.docker.io", name
        if "/" not in path:
            path = f"library/{path}"
    tag = "latest"
    if ":" in path.rsplit("/", 1)[-1]:
        path, tag = path.rsplit(":", 1)
    if registry == "docker.io":
        registry = "registry-1.docker.io"
    return ImageRef(registry, path, digest or tag)


MAX_CONFIG_OBJECT_SIZE = 2**22  # 4 MiB, as the reference


# -- registry documents (OCI image-spec manifest.md / config.md; Docker v2 schema 2) -----------
class _Doc(BaseModel):
    model_config = ConfigDict(extra="ignore", populate_by_name=True)


class Descriptor(_Doc):
    media_type: Optional[str] = Field(None, alias="mediaType")
    digest: str
    size: int = 0


class ImageManifest(_Doc):
    schema_version: int = Field(2, alias="schemaVersion")
    media_type: Optional[str] = Field(None, alias="mediaType")
    config: Descriptor
    layers: List[Descriptor] = []


class ImageConfigSection(_Doc):
    user: Optional[str] = Field(None, alias="User")
    entrypoint: Optional[List[str]] = Field(None, alias="Entrypoint")
    cmd: Optional[List[str]] = Field(None, alias="Cmd")
    env: Optional[List[str]] = Field(None, alias="Env")
    working_dir: Optional[str] = Field(None, alias="WorkingDir")

    @field_validator("user", mode="before")
    @classmethod
    def _empty_user(cls, v):
        return v or None  # "" means "whatever the runtime defaults to", i.e. unset


class ImageConfigObject(_Doc):
    architecture: Optional[str] = None
    os: Optional[str] = None
    config: ImageConfigSection = ImageConfigSection()

    @field_validator("config", mode="before")
    @classmethod
    def _null_config(cls, v):
        return {} if v is None else v  # `"config": null` is legal in the spec


def parse_image_manifest(obj: dict) -> ImageManifest:
    try:
        return ImageManifest.model_validate(obj)
    except ValueError as e:
        raise DockerRegistryError(f"malformed image manifest: {e}") from e


def parse_image_config_object(obj: dict) -> ImageConfig:
    try:
        c = ImageConfigObject.model_validate(obj).config
    except ValueError as e:
        raise DockerRegistryError(f"malformed image config: {e}") from e
    return ImageConfig(user=c.user, entrypoint=c.entrypoint, cmd=c.cmd, env=c.env or [])


def is_valid_docker_volume_target(path: str) -> bool:
    """A container mount target Docker accepts: absolute, no trailing slash (except ``/``), no NUL
    (reference: ``S/services/docker.py:155-163``)."""
    if not path.startswith("/") or "\0" in path:
        return False
    return path == "/" or not path.endswith("/")


class RegistryClient:
    def __init__(self, client: Optional[httpx.Client] = None):
        self.http = client or httpx.Client(timeout=30, follow_redirects=True)
        self._cache: Dict[Tuple[str, Optional[str]], Tuple[float, ImageConfig]] = {}
        self._lock = threading.Lock()

    def _token(self, challenge: str, auth: Optional[Tuple[str, str]]) -> Optional[str]:
        params = dict(p.split("=", 1) for p in challenge[len("Bearer "):].replace('"', "").split(","))
        realm = params.pop("realm")
        r = self.http.get(realm, params=params, auth=auth)
        if r.status_code != 200:
            return None
        d = r.json()
        return d.get("token") or d.get("access_token")

    def _get(self, url: str, headers: dict, auth, state: dict) -> httpx.Response:
        if state.get("token"):
            headers = {**headers, "Authorization": f"Bearer {state['token']}"}
        r = self.http.get(url, headers=headers, auth=auth if not state.get("token") else None)
        if r.status_code == 401 and r.headers.get("www-authenticate", "").startswith("Bearer "):
            state["token"] = self._token(r.headers["www-authenticate"], auth)
            if state["token"]:
                r = self.http.get(url, headers={**headers, "Authorization": f"Bearer {state['token']}"})
        return r

    def get_image_config(self, image: str, username: Optional[str] = None,
                         password: Optional[str] = None) -> ImageConfig:
        key = (image, username)
        with self._lock:
            hit = self._cache.get(key)
            if hit and time.time() - hit[0] < CACHE_TTL:
                return hit[1]
        ref = parse_image_name(image)
        base = f"https://{ref.registry}/v2/{ref.repository}"
        auth = (username, password) if username and password else None
        state: dict = {}
        r = self._get(f"{base}/manifests/{ref.reference}", {"Accept": MANIFEST_TYPES}, auth, state)
        if r.status_code != 200:
            raise DockerRegistryError(f"manifest of {ref.repository}:{ref.reference}: HTTP {r.status_code}", r.status_code)
        m = r.json()
        if "manifests" in m:  # index: pick linux/amd64
            chosen = next((x for x in m["manifests"] if x.get("platform", {}).get("os") == "linux"
                           and x.get("platform", {}).get("architecture") == "amd64"), m["manifests"][0])
            r = self._get(f"{base}/manifests/{chosen['digest']}", {"Accept": MANIFEST_TYPES}, auth, state)
            if r.status_code != 200:
                raise DockerRegistryError(f"platform manifest: HTTP {r.status_code}", r.status_code)
            m = r.json()
        digest = parse_image_manifest(m).config.digest
        headers = {"Authorization": f"Bearer {state['token']}"} if state.get("token") else {}
        with self.http.stream("GET", f"{base}/blobs/{digest}", headers=headers,
                              auth=None if state.get("token") else auth) as r:
            if r.status_code != 200:
                raise DockerRegistryError(f"config blob: HTTP {r.status_code}", r.status_code)
            body = join_byte_stream_checked(r.iter_bytes(), MAX_CONFIG_OBJECT_SIZE)  # stop reading past the cap
        if body is None:
            raise DockerRegistryError(f"image config object exceeds the size limit of {MAX_CONFIG_OBJECT_SIZE} bytes")
        try:
            obj = json.loads(body)
        except ValueError as e:
            raise DockerRegistryError(f"malformed image config: {e}") from e
        cfg = parse_image_config_object(obj)
        with self._lock:
            self._cache[key] = (time.time(), cfg)
        return cfg


_client: Optional[RegistryClient] = None


def get_image_config(image: str, username: Optional[str] = None, password: Optional[str] = None) -> ImageConfig:
    global _client
    if _client is None:
        _client = RegistryClient()
    return _client.get_image_config(image, username, password)
