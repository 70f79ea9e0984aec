"""Environment variables in run configurations (reference: ``C/models/envs.py:13-60``).

Accepts a mapping or a list of ``KEY=VALUE`` / ``KEY`` strings; a bare ``KEY`` is a sentinel that
is filled from the client's environment at apply time (e.g. ``- HF_TOKEN``).
"""

from __future__ import annotations

import re
from typing import Any, Dict, Iterator, List, Mapping, Union

from pydantic import GetCoreSchemaHandler
from pydantic_core import core_schema

_ENV_RE = re.compile(r"^([a-zA-Z_][a-zA-Z0-9_]*)(=.*$|$)")


class EnvSentinel:
    """Placeholder for a variable whose value comes from the client environment."""

    def __init__(self, key: str):
        self.key = key

    def from_env(self, env: Mapping[str, str]) -> str:
        if self.key in env:
            return env[self.key]
        raise ValueError(f"Environment variable {self.key} is not set")

    def __eq__(self, other):
        return isinstance(other, EnvSentinel) and other.key == self.key

    def __repr__(self):
        return f"EnvSentinel({self.key})"


class Env:
    def __init__(self, data: Union[None, Dict[str, Any], List[str], "Env"] = None):
        self._d: Dict[str, Union[str, EnvSentinel]] = {}
        if data is None:
            return
        if isinstance(data, Env):
            self._d = dict(data._d)
        elif isinstance(data, list):
            for var in data:
                if not isinstance(var, str) or not _ENV_RE.match(var):
                    raise ValueError(f"Invalid environment variable: {var!r}")
                if "=" in var:
                    k, v = var.split("=", 1)
                else:
                    k, v = var, EnvSentinel(var)
                if k in self._d:
                    raise ValueError(f"Duplicate environment variable: {var}")
                self._d[k] = v
        elif isinstance(data, dict):
            for k, v in data.items():
                if not isinstance(k, str) or not _ENV_RE.match(k):
                    raise ValueError(f"Invalid environment variable name: {k!r}")
                if isinstance(v, dict) and "key" in v:  # serialized sentinel
                    v = EnvSentinel(v["key"])
                elif v is None:
                    v = EnvSentinel(k)
                elif not isinstance(v, EnvSentinel):
                    v = str(v)
                self._d[k] = v
        else:
            raise ValueError(f"Invalid env: {data!r}")

    # mapping protocol
    def __iter__(self) -> Iterator[str]:
        return iter(self._d)

    def __contains__(self, k) -> bool:
        return k in self._d

    def __len__(self) -> int:
        return len(self._d)

    def __getitem__(self, k):
        return self._d[k]

    def __setitem__(self, k, v):
        self._d[k] = v

    def __eq__(self, other):
        return isinstance(other, Env) and other._d == self._d

    def __repr__(self):
        return f"Env({self._d})"

    def items(self):
        return self._d.items()

    def keys(self):
        return self._d.keys()

    def update(self, other):
        for k, v in (other.items() if hasattr(other, "items") else other):
            self._d[k] = v

    def resolve(self, environ: Mapping[str, str]) -> "Env":
        """Fill sentinels from ``environ`` (client side)."""
        return Env({k: (v.from_env(environ) if isinstance(v, EnvSentinel) else v) for k, v in self._d.items()})

    def as_dict(self) -> Dict[str, str]:
        unresolved = sorted(k for k, v in self._d.items() if isinstance(v, EnvSentinel))
        if unresolved:
            raise ValueError(f"Unresolved environment variables: {', '.join(unresolved)}")
        return dict(self._d)  # type: ignore[arg-type]

    def to_json(self) -> Dict[str, Any]:
        return {k: ({"key": v.key} if isinstance(v, EnvSentinel) else v) for k, v in self._d.items()}

    @classmethod
    def __get_pydantic_core_schema__(cls, source, handler: GetCoreSchemaHandler):
        return core_schema.no_info_plain_validator_function(
            lambda v: v if isinstance(v, Env) else Env(v),
            json_schema_input_schema=core_schema.union_schema(
                [core_schema.list_schema(core_schema.str_schema()), core_schema.dict_schema(core_schema.str_schema())]),
            serialization=core_schema.plain_serializer_function_ser_schema(
                lambda e: e.to_json(), return_schema=core_schema.dict_schema(core_schema.str_schema())),
        )
