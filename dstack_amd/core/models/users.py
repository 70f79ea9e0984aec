"""Users, roles, projects, members, secrets, server info (reference: ``C/models/users.py``,
``projects.py``, ``secrets.py``, ``server.py``)."""

from __future__ import annotations

import uuid
from datetime import datetime
from enum import Enum
from typing import List, Optional

from dstack_amd.core.models.backends import BackendInfo
from dstack_amd.core.models.common import CoreModel


class GlobalRole(str, Enum):
    ADMIN = "admin"
    USER = "user"


class ProjectRole(str, Enum):
    ADMIN = "admin"
    MANAGER = "manager"
    USER = "user"


class UserPermissions(CoreModel):
    can_create_projects: bool = True


class MemberPermissions(CoreModel):
    can_manage_ssh_fleets: bool = True


class User(CoreModel):
    id: uuid.UUID
    username: str
    created_at: Optional[datetime] = None
    global_role: GlobalRole
    email: Optional[str] = None
    active: bool = True
    permissions: UserPermissions = UserPermissions()


class UserTokenCreds(CoreModel):
    token: str


class UserWithCreds(User):
    creds: UserTokenCreds


class Member(CoreModel):
    user: User
    project_role: ProjectRole
    permissions: MemberPermissions = MemberPermissions()


class Project(CoreModel):
    project_id: uuid.UUID
    project_name: str
    owner: User
    created_at: Optional[datetime] = None
    backends: List[BackendInfo] = []
    members: List[Member] = []


class Secret(CoreModel):
    name: str
    value: Optional[str] = None


class ServerInfo(CoreModel):
    server_version: Optional[str] = None
