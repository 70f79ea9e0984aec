"""``user:group`` parsing for run containers (reference: ``C/models/unix.py``)."""

from __future__ import annotations

import re
from typing import Optional, Union

from dstack_amd.core.models.common import CoreModel


class UnixUser(CoreModel):
    uid: Optional[int] = None
    username: Optional[str] = None
    gid: Optional[int] = None
    groupname: Optional[str] = None

    @classmethod
    def parse(cls, v: str) -> "UnixUser":
        """``user[:group]``, each a name or a numeric id (reference ``UnixUser.parse``)."""
        parts = v.split(":")
        if len(parts) > 2:
            raise ValueError(f"invalid user: {v!r}: too many parts (expected user[:group])")
        user, group = parts[0], (parts[1] if len(parts) == 2 else None)
        if not user:
            raise ValueError(f"invalid user: {v!r}: empty user name or id")
        if group is not None and not group:
            raise ValueError(f"invalid user: {v!r}: empty group name or id")
        kw: dict = {}
        if re.fullmatch(r"-?\d+", user):
            if int(user) < 0:
                raise ValueError(f"invalid user: {v!r}: negative uid")
            kw["uid"] = int(user)
        else:
            kw["username"] = user
        if group is not None:
            if re.fullmatch(r"-?\d+", group):
                if int(group) < 0:
                    raise ValueError(f"invalid user: {v!r}: negative gid")
                kw["gid"] = int(group)
            else:
                kw["groupname"] = group
        return cls(**kw)

    def __str__(self) -> str:
        u: Union[int, str, None] = self.username if self.username is not None else self.uid
        g: Union[int, str, None] = self.groupname if self.groupname is not None else self.gid
        return f"{u}:{g}" if g is not None else str(u)
