"""Optional object storage for code blobs (reference: ``S/services/storage.py:13-74``, S3).

``DSTACK_SERVER_S3_BUCKET`` would enable S3 in the reference; boto3 is not available in this
image, so the MI355X build ships a filesystem store (``DSTACK_SERVER_CODE_STORE_DIR``) with the
same interface; when neither is set, blobs stay in the database."""

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


def get_default_storage() -> Optional[FileStorage]:
    d = os.getenv("DSTACK_SERVER_CODE_STORE_DIR")
    return FileStorage(d) if d else None
