"""Path helpers (reference: ``src/dstack/_internal/utils/path.py``)."""

from __future__ import annotations

from pathlib import PurePath, PurePosixPath
from typing import Union


def resolve_relative_path(path: Union[str, PurePath]) -> PurePath:
    """Normalise a path relative to the repo root (``a/./../b`` -> ``b``); absolute paths and
    paths that climb out of the repo are errors."""
    p = PurePosixPath(path)
    if p.is_absolute():
        raise ValueError(f"path must be relative: {path}")
    out = []
    for part in p.parts:
        if part in ("", "."):
            continue
        if part == "..":
            if not out:
                raise ValueError(f"path escapes the repository: {path}")
            out.pop()
        else:
            out.append(part)
    return PurePosixPath(*out) if out else PurePosixPath(".")
