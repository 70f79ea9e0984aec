"""Optional object storage for code blobs (reference: ``S/services/storage.py:13-74``, S3).

* ``DSTACK_SERVER_S3_BUCKET``: S3 over its REST API with SigV4 (no boto3), key
  ``data/projects/{project}/codes/{repo_id}/{blob_hash}`` as in the reference;
* ``DSTACK_SERVER_CODE_STORE_DIR``: the same layout on a (shared) filesystem;
* neither: blobs stay in the database."""

from __future__ import annotations

import os
from pathlib import Path
from typing import Optional


class FileStorage:
    def __init__(self, root: str):
        self.root = Path(root)

    def _path(self, project: str, repo_id: str, blob_hash: str) -> Path:
        return self.root / "data" / "projects" / project / "codes" / repo_id / blob_hash

    def upload_code(self, project: str, repo_id: str, blob_hash: str, blob: bytes):
        p = self._path(project, repo_id, blob_hash)
        p.parent.mkdir(parents=True, exist_ok=True)
        tmp = p.with_suffix(".tmp")
        tmp.write_bytes(blob)
        tmp.replace(p)

    def get_code(self, project: str, repo_id: str, blob_hash: str) -> bytes:
        p = self._path(project, repo_id, blob_hash)
        return p.read_bytes() if p.exists() else b""


class S3Storage:
    def __init__(self, bucket: str, region: Optional[str] = None, client=None, endpoint: Optional[str] = None):
        import httpx

        self.bucket = bucket
        from dstack_amd.server import settings

        self.region = region or settings.SERVER_BUCKET_REGION or os.getenv("AWS_REGION", "us-east-1")
        self.endpoint = endpoint or f"https://{bucket}.s3.{self.region}.amazonaws.com"
        self.http = client or httpx.Client(timeout=60)
        self.access_key = os.getenv("AWS_ACCESS_KEY_ID", "")
        self.secret_key = os.getenv("AWS_SECRET_ACCESS_KEY", "")
        self.token = os.getenv("AWS_SESSION_TOKEN")

    @staticmethod
    def _key(project: str, repo_id: str, blob_hash: str) -> str:
        return f"data/projects/{project}/codes/{repo_id}/{blob_hash}"

    def _req(self, method: str, key: str, body: bytes = b""):
        from dstack_amd.core.backends.clouds.common import sigv4_headers

        url = f"{self.endpoint}/{key}"
        h = sigv4_headers(method, url, self.region, "s3", self.access_key, self.secret_key, body, self.token)
        return self.http.request(method, url, content=body or None, headers=h)

    def upload_code(self, project: str, repo_id: str, blob_hash: str, blob: bytes):
        r = self._req("PUT", self._key(project, repo_id, blob_hash), blob)
        if r.status_code >= 300:
            raise RuntimeError(f"S3 put failed: {r.status_code} {r.text[:200]}")

    def get_code(self, project: str, repo_id: str, blob_hash: str) -> bytes:
        r = self._req("GET", self._key(project, repo_id, blob_hash))
        if r.status_code == 404:
            return b""
        if r.status_code >= 300:
            raise RuntimeError(f"S3 get failed: {r.status_code} {r.text[:200]}")
        return r.content


def get_default_storage():
    bucket = os.getenv("DSTACK_SERVER_BUCKET") or os.getenv("DSTACK_SERVER_S3_BUCKET")
    if bucket:
        return S3Storage(bucket)
    d = os.getenv("DSTACK_SERVER_CODE_STORE_DIR")
    return FileStorage(d) if d else None
