"""Projects and members (reference: ``S/services/projects.py``)."""

from __future__ import annotations

import json
import uuid
from typing import List, Optional

from sqlalchemy import select
from sqlalchemy.orm import Session

from dstack_amd.core.errors import ForbiddenError, ResourceExistsError, ResourceNotExistsError, ServerClientError
from dstack_amd.core.models.backends import BackendInfo, BackendType
from dstack_amd.core.models.users import GlobalRole, Member, Project, ProjectRole
from dstack_amd.server.models import MemberModel, ProjectModel, UserModel
from dstack_amd.server.services.permissions import check_can_create_projects, get_member_permissions
from dstack_amd.server.services.users import get_user_by_name, user_model_to_user
from dstack_amd.utils.common import generate_rsa_key_pair


def project_model_to_project(p: ProjectModel, include_backends: bool = True) -> Project:
    members = [Member(user=user_model_to_user(m.user), project_role=ProjectRole(m.project_role),
                      permissions=get_member_permissions(m)) for m in p.members]
    backends = []
    if include_backends:
        # settings only: credentials live in the encrypted auth column and are never returned
        backends = [BackendInfo(name=BackendType(b.type), config=json.loads(b.config or "{}")) for b in p.backends]
    return Project(project_id=p.id, project_name=p.name, owner=user_model_to_user(p.owner), created_at=p.created_at,
                   backends=backends, members=members)


def get_project_by_name(s: Session, name: str, include_deleted: bool = False) -> Optional[ProjectModel]:
    q = select(ProjectModel).where(ProjectModel.name == name)
    if not include_deleted:
        q = q.where(ProjectModel.deleted == False)  # noqa: E712
    return s.execute(q).scalar_one_or_none()


def get_project_or_error(s: Session, name: str) -> ProjectModel:
    p = get_project_by_name(s, name)
    if p is None:
        raise ResourceNotExistsError(f"Project {name} not found")
    return p


def list_user_projects(s: Session, user: UserModel) -> List[ProjectModel]:
    projects = list(s.execute(select(ProjectModel).where(ProjectModel.deleted == False)).scalars())  # noqa: E712
    if user.global_role == GlobalRole.ADMIN.value:
        return projects
    return [p for p in projects if any(m.user_id == user.id for m in p.members)]


def create_project(s: Session, user: UserModel, project_name: str) -> ProjectModel:
    check_can_create_projects(user)
    if user.global_role != GlobalRole.ADMIN.value:
        owned = s.execute(select(ProjectModel).where(ProjectModel.owner_id == user.id,
                                                     ProjectModel.deleted == False)).scalars().all()  # noqa: E712
        if len(owned) >= (user.projects_quota or 0):
            raise ServerClientError("User project quota exceeded")
    if get_project_by_name(s, project_name, include_deleted=True) is not None:
        raise ResourceExistsError(f"Project {project_name} exists")
    if not project_name.replace("-", "").replace("_", "").isalnum():
        raise ServerClientError("Project name may contain only letters, digits, - and _")
    private, public = generate_rsa_key_pair(f"dstack-{project_name}")
    p = ProjectModel(id=uuid.uuid4(), name=project_name, owner_id=user.id, ssh_private_key=private,
                     ssh_public_key=public)
    s.add(p)
    s.flush()
    add_member(s, p, user, ProjectRole.ADMIN)
    s.refresh(p)
    return p


def add_member(s: Session, project: ProjectModel, user: UserModel, role: ProjectRole):
    for m in project.members:
        if m.user_id == user.id:
            m.project_role = role.value
            return
    s.add(MemberModel(id=uuid.uuid4(), project_id=project.id, user_id=user.id, project_role=role.value,
                      member_num=len(project.members)))
    s.flush()


def set_members(s: Session, actor: UserModel, project: ProjectModel, members: List[dict]):
    role = get_member_role(project, actor)
    if actor.global_role != GlobalRole.ADMIN.value and role not in (ProjectRole.ADMIN, ProjectRole.MANAGER):
        raise ForbiddenError()
    if actor.global_role != GlobalRole.ADMIN.value and role == ProjectRole.MANAGER:
        # a manager manages users and managers, never the project's admins
        want = {(m["username"], ProjectRole(m["project_role"])) for m in members
                if ProjectRole(m["project_role"]) == ProjectRole.ADMIN}
        have = {(m.user.name, ProjectRole.ADMIN) for m in project.members
                if ProjectRole(m.project_role) == ProjectRole.ADMIN}
        if want != have:
            raise ForbiddenError("Access denied: changing project admins")
    for m in list(project.members):
        s.delete(m)
    s.flush()
    for i, m in enumerate(members):
        u = get_user_by_name(s, m["username"])
        if u is None:
            raise ResourceNotExistsError(f"User {m['username']} not found")
        s.add(MemberModel(id=uuid.uuid4(), project_id=project.id, user_id=u.id,
                          project_role=ProjectRole(m["project_role"]).value, member_num=i))
    s.flush()
    s.refresh(project)


def get_member_role(project: ProjectModel, user: UserModel) -> Optional[ProjectRole]:
    for m in project.members:
        if m.user_id == user.id:
            return ProjectRole(m.project_role)
    return None


def delete_projects(s: Session, actor: UserModel, names: List[str]):
    """Project admins delete their projects, global admins any; a regular user cannot delete every
    project they belong to (reference ``services/projects.py:delete_projects``)."""
    projects = [get_project_or_error(s, name) for name in names]
    if actor.global_role != GlobalRole.ADMIN.value:
        for p in projects:
            if get_member_role(p, actor) != ProjectRole.ADMIN:
                raise ForbiddenError()
        own = {p.id for p in list_user_projects(s, actor)}
        if own and own <= {p.id for p in projects}:
            raise ServerClientError("Cannot delete the only project")
    for p in projects:
        p.deleted = True
        p.name = f"_deleted_{p.id.hex[:8]}_{p.name}"[:50]


def get_or_create_default_project(s: Session, user: UserModel, name: str) -> ProjectModel:
    p = get_project_by_name(s, name)
    if p is None:
        p = create_project(s, user, name)
    return p
