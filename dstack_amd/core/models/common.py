"""Base model and small value types (reference: ``C/models/common.py``).

``CoreModel`` is pydantic v2: requests/configs are parsed with ``extra="forbid"`` (typos in YAML are
errors) while objects received from a newer server are parsed leniently via ``parse_lenient``.
"""

from __future__ import annotations

import re
from enum import Enum
from typing import Any, Optional, Type, TypeVar, Union

from pydantic import BaseModel, ConfigDict, GetCoreSchemaHandler
from pydantic_core import core_schema

M = TypeVar("M", bound="CoreModel")


class CoreModel(BaseModel):
    model_config = ConfigDict(extra="forbid", populate_by_name=True, use_enum_values=False,
                              protected_namespaces=())

    def json_dict(self, **kw) -> dict:
        return self.model_dump(mode="json", **kw)

    @classmethod
    def parse_lenient(cls: Type[M], data: Any) -> M:
        """Parse ignoring unknown fields (forward compatibility with newer peers)."""
        return _lenient(cls).model_validate(data)


_LENIENT_CACHE: dict = {}


def _lenient(cls):
    if cls not in _LENIENT_CACHE:
        _LENIENT_CACHE[cls] = type(
            cls.__name__, (cls,), {"model_config": ConfigDict(**{**cls.model_config, "extra": "ignore"})}
        )
    return _LENIENT_CACHE[cls]


_DURATION_RE = re.compile(r"^(\d+)\s*([smhdw])$")
_DURATION_UNITS = {"s": 1, "m": 60, "h": 3600, "d": 24 * 3600, "w": 7 * 24 * 3600}


class Duration(int):
    """Seconds; parses ``90``, ``"90"``, ``"5m"``, ``"2h"``, ``"1d"``, ``"1w"``."""

    @classmethod
    def parse(cls, v: Union[int, str, "Duration"]) -> "Duration":
        if isinstance(v, bool):
            raise ValueError(f"Invalid duration: {v}")
        if isinstance(v, int):
            return cls(v)
        if isinstance(v, str):
            s = v.strip().lower()
            if s.isdigit():
                return cls(int(s))
            m = _DURATION_RE.match(s)
            if m:
                return cls(int(m.group(1)) * _DURATION_UNITS[m.group(2)])
        raise ValueError(f"Invalid duration: {v!r}")

    @classmethod
    def __get_pydantic_core_schema__(cls, source, handler: GetCoreSchemaHandler):
        return core_schema.no_info_plain_validator_function(
            cls.parse,
            json_schema_input_schema=core_schema.union_schema([core_schema.int_schema(), core_schema.str_schema()]),
            serialization=core_schema.plain_serializer_function_ser_schema(int, return_schema=core_schema.int_schema()),
        )


def format_duration(seconds: Optional[int]) -> str:
    if seconds is None:
        return "-"
    for unit, n in (("w", 7 * 86400), ("d", 86400), ("h", 3600), ("m", 60)):
        if seconds >= n and seconds % n == 0:
            return f"{seconds // n}{unit}"
    return f"{seconds}s"


class RegistryAuth(CoreModel):
    """Credentials for pulling a private Docker image (hashable: a cache key of the registry
    client's image-config cache)."""

    username: str
    password: str

    def __hash__(self) -> int:
        return hash((self.username, self.password))


class ApplyAction(str, Enum):
    CREATE = "create"
    UPDATE = "update"


class NetworkMode(str, Enum):
    HOST = "host"
    BRIDGE = "bridge"
