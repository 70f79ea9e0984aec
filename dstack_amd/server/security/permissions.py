"""Auth dependencies (reference: ``S/security/permissions.py:23-124``): Bearer token -> user;
role checks ``Authenticated``, ``GlobalAdmin``, ``ProjectAdmin``, ``ProjectManager``,
``ProjectMember``."""

from __future__ import annotations

from typing import Tuple

from fastapi import Depends, Request
from sqlalchemy.orm import Session

from dstack_amd.core.errors import ForbiddenError, ResourceNotExistsError, UnauthorizedError
from dstack_amd.core.models.users import GlobalRole, ProjectRole
from dstack_amd.server.deps import get_session
from dstack_amd.server.models import ProjectModel, UserModel
from dstack_amd.server.services import projects as projects_services
from dstack_amd.server.services.users import get_user_by_token


def _token(request: Request) -> str:
    auth = request.headers.get("authorization", "")
    if not auth.lower().startswith("bearer "):
        raise UnauthorizedError()
    return auth[7:].strip()


def authenticated(request: Request, s: Session = Depends(get_session, scope="function")) -> UserModel:
    user = get_user_by_token(s, _token(request))
    if user is None or not user.active:
        raise UnauthorizedError()
    return user


def global_admin(user: UserModel = Depends(authenticated)) -> UserModel:
    if user.global_role != GlobalRole.ADMIN.value:
        raise ForbiddenError()
    return user


def _project_access(project_name: str, user: UserModel, s: Session, roles) -> Tuple[UserModel, ProjectModel]:
    project = projects_services.get_project_by_name(s, project_name)
    if project is None:
        raise ResourceNotExistsError(f"Project {project_name} not found")
    if user.global_role == GlobalRole.ADMIN.value:
        return user, project
    role = projects_services.get_member_role(project, user)
    if role is None or role not in roles:
        raise ForbiddenError()
    return user, project


def project_member(project_name: str, user: UserModel = Depends(authenticated),
                   s: Session = Depends(get_session, scope="function")) -> Tuple[UserModel, ProjectModel]:
    return _project_access(project_name, user, s, (ProjectRole.ADMIN, ProjectRole.MANAGER, ProjectRole.USER))


def project_manager(project_name: str, user: UserModel = Depends(authenticated),
                    s: Session = Depends(get_session, scope="function")) -> Tuple[UserModel, ProjectModel]:
    return _project_access(project_name, user, s, (ProjectRole.ADMIN, ProjectRole.MANAGER))


def project_admin(project_name: str, user: UserModel = Depends(authenticated),
                  s: Session = Depends(get_session, scope="function")) -> Tuple[UserModel, ProjectModel]:
    return _project_access(project_name, user, s, (ProjectRole.ADMIN,))
