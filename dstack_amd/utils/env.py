"""Environment variable helpers (reference: ``src/dstack/_internal/utils/env.py``)."""

from __future__ import annotations

import os

_TRUE = {"1", "true", "yes", "on"}
_FALSE = {"0", "false", "no", "off"}


def get_bool(name: str, default: bool = False) -> bool:
    """``name`` as a boolean: unset -> ``default``; 1/true/yes/on and 0/false/no/off in any case;
    anything else (the empty string included) is a configuration error naming the variable."""
    v = os.environ.get(name)
    if v is None:
        return default
    low = v.strip().lower()
    if low in _TRUE:
        return True
    if low in _FALSE:
        return False
    raise ValueError(f"invalid boolean in environment: {name}={v}")
