"""Users and tokens (reference: ``S/services/users.py``)."""

from __future__ import annotations

import uuid
from typing import List, Optional

from sqlalchemy import select
from sqlalchemy.orm import Session

from dstack_amd.core.errors import ForbiddenError, ResourceExistsError, ResourceNotExistsError
from dstack_amd.core.models.users import GlobalRole, User, UserTokenCreds, UserWithCreds
from dstack_amd.server.models import UserModel
from dstack_amd.utils.common import generate_token, token_hash


def user_model_to_user(u: UserModel) -> User:
    from dstack_amd.server.services.permissions import get_user_permissions

    return User(id=u.id, username=u.name, created_at=u.created_at, global_role=GlobalRole(u.global_role),
                email=u.email, active=u.active, permissions=get_user_permissions(u))


def user_model_to_user_with_creds(u: UserModel) -> UserWithCreds:
    return UserWithCreds(**user_model_to_user(u).model_dump(), creds=UserTokenCreds(token=u.token))


def get_user_by_name(s: Session, name: str) -> Optional[UserModel]:
    return s.execute(select(UserModel).where(UserModel.name == name)).scalar_one_or_none()


def get_user_by_token(s: Session, token: str) -> Optional[UserModel]:
    return s.execute(select(UserModel).where(UserModel.token_hash == token_hash(token))).scalar_one_or_none()


def list_users(s: Session) -> List[UserModel]:
    return list(s.execute(select(UserModel).order_by(UserModel.created_at)).scalars())


def create_user(s: Session, username: str, global_role: GlobalRole = GlobalRole.USER, email: Optional[str] = None,
                token: Optional[str] = None, active: bool = True) -> UserModel:
    if get_user_by_name(s, username) is not None:
        raise ResourceExistsError(f"User {username} exists")
    token = token or generate_token()
    from dstack_amd.server import settings

    u = UserModel(id=uuid.uuid4(), name=username, token=token, token_hash=token_hash(token),
                  global_role=global_role.value, email=email, active=active,
                  projects_quota=settings.USER_PROJECT_DEFAULT_QUOTA)
    s.add(u)
    s.flush()
    return u


def update_user(s: Session, username: str, global_role: GlobalRole, email: Optional[str] = None,
                active: Optional[bool] = None) -> UserModel:
    u = get_user_by_name(s, username)
    if u is None:
        raise ResourceNotExistsError()
    u.global_role = global_role.value
    if email is not None:
        u.email = email
    if active is not None:
        u.active = active
    return u


def refresh_token(s: Session, actor: UserModel, username: str) -> UserModel:
    if actor.global_role != GlobalRole.ADMIN.value and actor.name != username:
        raise ForbiddenError()
    u = get_user_by_name(s, username)
    if u is None:
        raise ResourceNotExistsError()
    token = generate_token()
    u.token = token
    u.token_hash = token_hash(token)
    return u


def delete_users(s: Session, actor: UserModel, usernames: List[str]):
    if actor.global_role != GlobalRole.ADMIN.value:
        raise ForbiddenError()
    for name in usernames:
        u = get_user_by_name(s, name)
        if u is not None:
            s.delete(u)


def get_or_create_admin_user(s: Session, token: Optional[str] = None) -> UserModel:
    u = get_user_by_name(s, "admin")
    if u is None:
        u = create_user(s, "admin", GlobalRole.ADMIN, token=token)
    elif token and u.token != token:
        u.token = token
        u.token_hash = token_hash(token)
    return u
