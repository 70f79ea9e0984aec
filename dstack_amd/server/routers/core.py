"""REST routers: server, users, projects, backends, secrets, repos (reference:
``S/routers/{server,users,projects,backends,secrets,repos}.py``).  All JSON ``POST``."""

from __future__ import annotations

import os
from typing import List, Tuple

import yaml
from fastapi import APIRouter, Depends, Request
from sqlalchemy.orm import Session

from dstack_amd import __version__
from dstack_amd.core.errors import ForbiddenError, RepoDoesNotExistError, ResourceNotExistsError, ServerClientError
from dstack_amd.core.models.repos import RepoHead
from dstack_amd.core.models.users import GlobalRole, Project, ServerInfo, User, UserWithCreds
from dstack_amd.server import schemas
from dstack_amd.server.deps import get_session
from dstack_amd.server.models import ProjectModel, UserModel
from dstack_amd.server.security.permissions import (
    authenticated,
    global_admin,
    project_admin,
    project_manager,
    project_member,
)
from dstack_amd.server.services import backends as backends_services
from dstack_amd.server.services import projects as projects_services
from dstack_amd.server.services import repos as repos_services
from dstack_amd.server.services import secrets as secrets_services
from dstack_amd.server.services import users as users_services

server_router = APIRouter(prefix="/api/server", tags=["server"])
users_router = APIRouter(prefix="/api/users", tags=["users"])
projects_router = APIRouter(prefix="/api/projects", tags=["projects"])
backends_router = APIRouter(prefix="/api/backends", tags=["backends"])
project_backends_router = APIRouter(prefix="/api/project/{project_name}/backends", tags=["backends"])
secrets_router = APIRouter(prefix="/api/project/{project_name}/secrets", tags=["secrets"])
repos_router = APIRouter(prefix="/api/project/{project_name}/repos", tags=["repos"])

UP = Tuple[UserModel, ProjectModel]


@server_router.post("/get_info")
def get_server_info() -> ServerInfo:
    return ServerInfo(server_version=__version__)


# ---- users ----------------------------------------------------------------------------------
@users_router.post("/list")
def list_users(user: UserModel = Depends(authenticated), s: Session = Depends(get_session, scope="function")) -> List[User]:
    if user.global_role != GlobalRole.ADMIN.value:
        return [users_services.user_model_to_user(user)]
    return [users_services.user_model_to_user(u) for u in users_services.list_users(s)]


@users_router.post("/get_my_user")
def get_my_user(user: UserModel = Depends(authenticated)) -> UserWithCreds:
    return users_services.user_model_to_user_with_creds(user)


@users_router.post("/get_user")
def get_user(body: schemas.GetUserRequest, user: UserModel = Depends(authenticated),
             s: Session = Depends(get_session, scope="function")) -> UserWithCreds:
    if user.global_role != GlobalRole.ADMIN.value and user.name != body.username:
        raise ForbiddenError()
    u = users_services.get_user_by_name(s, body.username)
    if u is None:
        raise ResourceNotExistsError()
    return users_services.user_model_to_user_with_creds(u)


@users_router.post("/create")
def create_user(body: schemas.CreateUserRequest, user: UserModel = Depends(global_admin),
                s: Session = Depends(get_session, scope="function")) -> UserWithCreds:
    u = users_services.create_user(s, body.username, body.global_role, body.email, active=body.active)
    return users_services.user_model_to_user_with_creds(u)


@users_router.post("/update")
def update_user(body: schemas.UpdateUserRequest, user: UserModel = Depends(global_admin),
                s: Session = Depends(get_session, scope="function")) -> User:
    return users_services.user_model_to_user(
        users_services.update_user(s, body.username, body.global_role, body.email, body.active))


@users_router.post("/refresh_token")
def refresh_token(body: schemas.RefreshTokenRequest, user: UserModel = Depends(authenticated),
                  s: Session = Depends(get_session, scope="function")) -> UserWithCreds:
    return users_services.user_model_to_user_with_creds(users_services.refresh_token(s, user, body.username))


@users_router.post("/delete")
def delete_users(body: schemas.DeleteUsersRequest, user: UserModel = Depends(global_admin),
                 s: Session = Depends(get_session, scope="function")):
    users_services.delete_users(s, user, body.users)
    return {}


# ---- projects -------------------------------------------------------------------------------
@projects_router.post("/list")
def list_projects(user: UserModel = Depends(authenticated), s: Session = Depends(get_session, scope="function")) -> List[Project]:
    return [projects_services.project_model_to_project(p) for p in projects_services.list_user_projects(s, user)]


@projects_router.post("/create")
def create_project(body: schemas.CreateProjectRequest, user: UserModel = Depends(authenticated),
                   s: Session = Depends(get_session, scope="function")) -> Project:
    return projects_services.project_model_to_project(projects_services.create_project(s, user, body.project_name))


@projects_router.post("/delete")
def delete_projects(body: schemas.DeleteProjectsRequest, user: UserModel = Depends(authenticated),
                    s: Session = Depends(get_session, scope="function")):
    projects_services.delete_projects(s, user, body.projects_names)
    return {}


@projects_router.post("/{project_name}/get")
def get_project(up: UP = Depends(project_member)) -> Project:
    return projects_services.project_model_to_project(up[1])


@projects_router.post("/{project_name}/set_members")
def set_members(body: schemas.SetProjectMembersRequest, up: UP = Depends(project_manager),
                s: Session = Depends(get_session, scope="function")) -> Project:
    projects_services.set_members(s, up[0], up[1], [m.model_dump(mode="json") for m in body.members])
    return projects_services.project_model_to_project(up[1])


# ---- backends -------------------------------------------------------------------------------
@backends_router.post("/list_types")
def list_backend_types() -> List[str]:
    return backends_services.list_backend_types()


@backends_router.post("/config_values")
def backend_config_values(body: dict, user: UserModel = Depends(authenticated)) -> dict:
    """Choices for a backend form (reference ``/api/backends/config_values``): the regions the
    catalog knows for the type, with the requested ones (or all) selected; credentials are
    validated when the backend is created."""
    return backends_services.backend_config_values(body)


@backends_router.post("/form_schema")
def backend_form_schema(user: UserModel = Depends(authenticated)) -> dict:
    """Field descriptors of every configurable backend type (the web UI builds its forms from them)."""
    from dstack_amd.core.models.backend_configs import backend_form_schema as schema

    return schema()


@project_backends_router.post("/create")
def create_backend(body: dict, up: UP = Depends(project_admin), s: Session = Depends(get_session, scope="function")) -> dict:
    backends_services.create_backend(s, up[1], body)
    return body


@project_backends_router.post("/update")
def update_backend(body: dict, up: UP = Depends(project_admin), s: Session = Depends(get_session, scope="function")) -> dict:
    backends_services.update_backend(s, up[1], body)
    return body


@project_backends_router.post("/delete")
def delete_backends(body: schemas.DeleteBackendsRequest, up: UP = Depends(project_admin),
                    s: Session = Depends(get_session, scope="function")):
    backends_services.delete_backends(s, up[1], body.backends_names)
    return {}


@project_backends_router.post("/{backend_name}/config_info")
def backend_config_info(backend_name: str, up: UP = Depends(project_admin), s: Session = Depends(get_session, scope="function")) -> dict:
    return backends_services.backend_config_info(s, up[1], backend_name)


@project_backends_router.post("/create_yaml")
def create_backend_yaml(body: schemas.CreateBackendYAMLRequest, up: UP = Depends(project_admin),
                        s: Session = Depends(get_session, scope="function")):
    cfg = yaml.safe_load(body.config_yaml) or {}
    if not isinstance(cfg, dict):
        raise ServerClientError("backend YAML must be a mapping")
    backends_services.create_backend(s, up[1], cfg)
    return {}


@project_backends_router.post("/update_yaml")
def update_backend_yaml(body: schemas.CreateBackendYAMLRequest, up: UP = Depends(project_admin),
                        s: Session = Depends(get_session, scope="function")):
    backends_services.update_backend(s, up[1], yaml.safe_load(body.config_yaml) or {})
    return {}


@project_backends_router.post("/{backend_name}/get_yaml")
def get_backend_yaml(backend_name: str, up: UP = Depends(project_admin), s: Session = Depends(get_session, scope="function")) -> dict:
    return {"name": backend_name,
            "config_yaml": yaml.safe_dump(backends_services.backend_config_info(s, up[1], backend_name))}


# ---- secrets --------------------------------------------------------------------------------
@secrets_router.post("/list")
def list_secrets(up: UP = Depends(project_manager), s: Session = Depends(get_session, scope="function")):
    return secrets_services.list_secrets(s, up[1])


@secrets_router.post("/get")
def get_secret(body: schemas.GetSecretRequest, up: UP = Depends(project_manager), s: Session = Depends(get_session, scope="function")):
    return secrets_services.get_secret(s, up[1], body.name)


@secrets_router.post("/add")
def add_secret(body: schemas.AddSecretRequest, up: UP = Depends(project_manager), s: Session = Depends(get_session, scope="function")):
    return secrets_services.add_secret(s, up[1], body.name, body.value)


@secrets_router.post("/delete")
def delete_secrets(body: schemas.DeleteSecretsRequest, up: UP = Depends(project_manager),
                   s: Session = Depends(get_session, scope="function")):
    secrets_services.delete_secrets(s, up[1], body.secrets_names)
    return {}


# ---- repos ----------------------------------------------------------------------------------
@repos_router.post("/list")
def list_repos(up: UP = Depends(project_member), s: Session = Depends(get_session, scope="function")) -> List[RepoHead]:
    return repos_services.list_repos(s, up[1])


@repos_router.post("/get")
def get_repo(body: schemas.GetRepoRequest, up: UP = Depends(project_member), s: Session = Depends(get_session, scope="function")):
    head = repos_services.get_repo_head(s, up[1], up[0], body.repo_id, body.include_creds)
    if head is None:
        raise RepoDoesNotExistError()
    return head


@repos_router.post("/init")
def init_repo(body: schemas.InitRepoRequest, up: UP = Depends(project_member), s: Session = Depends(get_session, scope="function")):
    repos_services.init_repo(s, up[1], up[0], body.repo_id, body.repo_info, body.repo_creds)
    return {}


@repos_router.post("/delete")
def delete_repos(body: schemas.DeleteReposRequest, up: UP = Depends(project_manager),
                 s: Session = Depends(get_session, scope="function")):
    repos_services.delete_repos(s, up[1], body.repos_ids)
    return {}


CODE_UPLOAD_LIMIT = int(os.environ.get("DSTACK_SERVER_CODE_UPLOAD_LIMIT", 64 * 2**20))


@repos_router.post("/upload_code")
async def upload_code(request: Request, repo_id: str, up: UP = Depends(project_member)):
    import hashlib

    from starlette.concurrency import run_in_threadpool

    from dstack_amd.server.db import session_scope

    from dstack_amd.server.utils.common import ajoin_byte_stream_checked

    # the body is read up to the cap (plus multipart framing) and no further
    blob = await ajoin_byte_stream_checked(request.stream(), CODE_UPLOAD_LIMIT + 2**16)
    if blob is None:
        raise ServerClientError(f"Code blob exceeds {CODE_UPLOAD_LIMIT // 2**20} MiB; use a remote repo or .dstackignore")
    ctype = request.headers.get("content-type", "")
    if ctype.startswith("multipart/form-data"):
        # the reference client posts the tarball as the multipart field "file"
        from email.parser import BytesParser
        from email.policy import HTTP

        msg = BytesParser(policy=HTTP).parsebytes(b"Content-Type: " + ctype.encode() + b"\r\n\r\n" + blob)
        parts = [p for p in msg.iter_parts() if p.get_param("name", header="content-disposition") == "file"]
        if not parts:
            raise ServerClientError("multipart upload without a 'file' field")
        blob = parts[0].get_payload(decode=True) or b""
    if len(blob) > CODE_UPLOAD_LIMIT:
        raise ServerClientError(f"Code blob exceeds {CODE_UPLOAD_LIMIT // 2**20} MiB; use a remote repo or .dstackignore")
    blob_hash = hashlib.sha256(blob).hexdigest()
    project_id = up[1].id

    def store():
        with session_scope() as s:
            project = s.get(ProjectModel, project_id)
            repos_services.upload_code(s, project, repo_id, blob_hash, blob)

    await run_in_threadpool(store)
    return {"blob_hash": blob_hash}
