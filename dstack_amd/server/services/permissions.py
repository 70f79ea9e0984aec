"""Server-wide default permissions (``default_permissions`` of the server ``config.yml``) and the
per-user / per-member permissions derived from them (reference: ``S/services/permissions.py``,
``S/services/users.py:get_user_permissions``, ``S/services/projects.py:get_member_permissions``,
``S/services/fleets.py:_check_can_manage_ssh_fleets``).

* ``allow_non_admins_create_projects: false`` -- only global admins create projects.
* ``allow_non_admins_manage_ssh_fleets: false`` -- only global admins and project admins create
  or delete SSH fleets (on-prem hosts: adding one hands the project's users shell access to it).
"""

from __future__ import annotations

from typing import Optional

from dstack_amd.core.errors import ForbiddenError
from dstack_amd.core.models.common import CoreModel
from dstack_amd.core.models.users import GlobalRole, MemberPermissions, ProjectRole, UserPermissions


class DefaultPermissions(CoreModel):
    allow_non_admins_create_projects: bool = True
    allow_non_admins_manage_ssh_fleets: bool = True


_default = DefaultPermissions()


def get_default_permissions() -> DefaultPermissions:
    return _default


def set_default_permissions(p: Optional[DefaultPermissions]) -> None:
    global _default
    _default = p or DefaultPermissions()


def get_user_permissions(user) -> UserPermissions:
    admin = user.global_role == GlobalRole.ADMIN.value
    return UserPermissions(can_create_projects=admin or _default.allow_non_admins_create_projects)


def get_member_permissions(member) -> MemberPermissions:
    admin = member.user.global_role == GlobalRole.ADMIN.value or member.project_role == ProjectRole.ADMIN.value
    return MemberPermissions(can_manage_ssh_fleets=admin or _default.allow_non_admins_manage_ssh_fleets)


def check_can_create_projects(user) -> None:
    if not get_user_permissions(user).can_create_projects:
        raise ForbiddenError("Only global admins can create projects on this server")


def check_can_manage_ssh_fleets(user, project) -> None:
    if user is None or user.global_role == GlobalRole.ADMIN.value:
        return
    member = next((m for m in project.members if m.user_id == user.id), None)
    if member is None or not get_member_permissions(member).can_manage_ssh_fleets:
        raise ForbiddenError("Only global and project admins can manage SSH fleets in this project")
