"""``user:group`` parsing for run containers (reference: ``C/models/unix.py``)."""

from __future__ import annotations

from typing import Optional, Union

from dstack_amd.core.models.common import CoreModel


class UnixUser(CoreModel):
    uid: Optional[int] = None
    username: Optional[str] = None
    gid: Optional[int] = None
    groupname: Optional[str] = None

    @classmethod
    def parse(cls, v: str) -> "UnixUser":
        if not v:
            raise ValueError("empty user")
        parts = v.split(":")
        if len(parts) > 2:
            raise ValueError(f"invalid user: {v} (expected user[:group])")
        user, group = parts[0], (parts[1] if len(parts) == 2 else None)
        if not user or (group is not None and not group):
            raise ValueError(f"invalid user: {v}")
        if user.startswith("-") or (group or "").startswith("-"):
            raise ValueError(f"negative uid/gid: {v}")
        kw: dict = {}
        if user.isdigit():
            kw["uid"] = int(user)
        else:
            kw["username"] = user
        if group:
            if group.isdigit():
                kw["gid"] = int(group)
            else:
                kw["groupname"] = group
        return cls(**kw)

    def __str__(self) -> str:
        u: Union[int, str, None] = self.username if self.username is not None else self.uid
        g: Union[int, str, None] = self.groupname if self.groupname is not None else self.gid
        return f"{u}:{g}" if g is not None else str(u)
