"""Locate (and build on demand) the native agents: ``dstack-shim``, ``dstack-runner``,
``dstack-probe`` from ``native/`` (C++/HIP, built with ``make -C native``)."""

from __future__ import annotations

import os
import shutil
import subprocess
import threading
from pathlib import Path
from typing import Optional

REPO_ROOT = Path(__file__).resolve().parent.parent
NATIVE_DIR = REPO_ROOT / "native"
BUILD_DIR = NATIVE_DIR / "build"
_lock = threading.Lock()


def build_native(targets=("build/dstack-runner", "build/dstack-shim"), jobs: int = 8) -> None:
    with _lock:
        subprocess.run(["make", "-C", str(NATIVE_DIR), f"-j{jobs}", *targets], check=True, capture_output=True)


def binary_path(name: str, build_if_missing: bool = True) -> Optional[str]:
    env = os.environ.get(f"DSTACK_{name.upper().replace('-', '_')[7:]}_BINARY_PATH") if name.startswith("dstack-") else None
    if env and os.path.exists(env):
        return env
    p = BUILD_DIR / name
    if p.exists():
        return str(p)
    if build_if_missing and (NATIVE_DIR / "Makefile").exists() and shutil.which("make"):
        try:
            build_native((f"build/{name}",))
        except subprocess.CalledProcessError:
            return None
        if p.exists():
            return str(p)
    found = shutil.which(name)
    return found


def shim_path() -> Optional[str]:
    return binary_path("dstack-shim")


def runner_path() -> Optional[str]:
    return binary_path("dstack-runner")


def probe_path() -> Optional[str]:
    return binary_path("dstack-probe", build_if_missing=False)
