"""Repos and code blobs (reference: ``S/services/repos.py:37-362``, ``S/services/storage.py``)."""

from __future__ import annotations

import json
import uuid
from typing import List, Optional

from sqlalchemy import select
from sqlalchemy.orm import Session

from dstack_amd.core.errors import RepoDoesNotExistError
from dstack_amd.core.models.repos import (
    DEFAULT_VIRTUAL_REPO_ID,
    RemoteRepoCreds,
    RepoHead,
    RepoHeadWithCreds,
    VirtualRepoInfo,
)
from dstack_amd.server.models import CodeModel, ProjectModel, RepoCredsModel, RepoModel, UserModel


def get_repo(s: Session, project: ProjectModel, repo_id: str) -> Optional[RepoModel]:
    return s.execute(select(RepoModel).where(RepoModel.project_id == project.id,
                                             RepoModel.name == repo_id)).scalar_one_or_none()


def get_repo_or_error(s: Session, project: ProjectModel, repo_id: str) -> RepoModel:
    r = get_repo(s, project, repo_id)
    if r is None:
        raise RepoDoesNotExistError()
    return r


def get_or_create_virtual_repo(s: Session, project: ProjectModel, repo_id: str = DEFAULT_VIRTUAL_REPO_ID) -> RepoModel:
    r = get_repo(s, project, repo_id)
    if r is None:
        r = RepoModel(id=uuid.uuid4(), project_id=project.id, name=repo_id, type="virtual",
                      info=VirtualRepoInfo().model_dump_json())
        s.add(r)
        s.flush()
    return r


def repo_model_to_head(r: RepoModel, creds: Optional[dict] = None) -> RepoHeadWithCreds:
    return RepoHeadWithCreds.model_validate({
        "repo_id": r.name, "repo_info": json.loads(r.info),
        "repo_creds": creds,
    })


def get_repo_head(s: Session, project: ProjectModel, user: UserModel, repo_id: str,
                  include_creds: bool) -> Optional[RepoHeadWithCreds]:
    """The repo with the credentials the given user would clone it with: their own, else the
    repo's legacy shared ones, else none (reference: ``S/services/repos.py`` ``get_repo``)."""
    r = get_repo(s, project, repo_id)
    if r is None:
        return None
    return repo_model_to_head(r, get_repo_creds(s, r, user.id) if include_creds else None)


def list_repos(s: Session, project: ProjectModel) -> List[RepoHead]:
    rows = s.execute(select(RepoModel).where(RepoModel.project_id == project.id)).scalars()
    return [RepoHead.model_validate({"repo_id": r.name, "repo_info": json.loads(r.info)}) for r in rows]


def init_repo(s: Session, project: ProjectModel, user: UserModel, repo_id: str, repo_info: dict,
              repo_creds: Optional[dict]) -> RepoModel:
    r = get_repo(s, project, repo_id)
    if r is None:
        r = RepoModel(id=uuid.uuid4(), project_id=project.id, name=repo_id, type=repo_info.get("repo_type", "remote"),
                      info=json.dumps(repo_info))
        s.add(r)
        s.flush()
    else:
        r.info = json.dumps(repo_info)
        r.type = repo_info.get("repo_type", r.type)
    # the caller's own credentials are added, replaced, or -- when a remote repo is initialised
    # without them -- removed (reference ``init_repo``: creds are per user)
    c = s.execute(select(RepoCredsModel).where(RepoCredsModel.repo_id == r.id,
                                               RepoCredsModel.user_id == user.id)).scalar_one_or_none()
    if repo_creds is not None:
        RemoteRepoCreds.model_validate(repo_creds)
        if c is None:
            s.add(RepoCredsModel(id=uuid.uuid4(), repo_id=r.id, user_id=user.id, creds=json.dumps(repo_creds)))
        else:
            c.creds = json.dumps(repo_creds)
    elif c is not None and r.type == "remote":
        s.delete(c)
    return r


def get_repo_creds(s: Session, repo: RepoModel, user_id) -> Optional[dict]:
    c = s.execute(select(RepoCredsModel).where(RepoCredsModel.repo_id == repo.id,
                                               RepoCredsModel.user_id == user_id)).scalar_one_or_none()
    if c is not None:
        return json.loads(c.creds)
    if repo.creds:
        return json.loads(repo.creds)
    return None


def delete_repos(s: Session, project: ProjectModel, repo_ids: List[str]):
    for rid in repo_ids:
        r = get_repo(s, project, rid)
        if r is not None:
            s.delete(r)


def upload_code(s: Session, project: ProjectModel, repo_id: str, blob_hash: str, blob: bytes) -> CodeModel:
    repo = get_repo_or_error(s, project, repo_id)
    c = s.execute(select(CodeModel).where(CodeModel.repo_id == repo.id,
                                          CodeModel.blob_hash == blob_hash)).scalar_one_or_none()
    if c is None:
        from dstack_amd.server.services.storage import get_default_storage

        storage = get_default_storage()
        if storage is not None:
            storage.upload_code(project.name, repo_id, blob_hash, blob)
            c = CodeModel(id=uuid.uuid4(), repo_id=repo.id, blob_hash=blob_hash, blob=None)
        else:
            c = CodeModel(id=uuid.uuid4(), repo_id=repo.id, blob_hash=blob_hash, blob=blob)
        s.add(c)
        s.flush()
    return c


def get_code_blob(s: Session, project: ProjectModel, repo: RepoModel, blob_hash: Optional[str]) -> bytes:
    if not blob_hash:
        return b""
    c = s.execute(select(CodeModel).where(CodeModel.repo_id == repo.id,
                                          CodeModel.blob_hash == blob_hash)).scalar_one_or_none()
    if c is None:
        return b""
    if c.blob is None:
        from dstack_amd.server.services.storage import get_default_storage

        storage = get_default_storage()
        return storage.get_code(project.name, repo.name, blob_hash) if storage else b""
    return c.blob
