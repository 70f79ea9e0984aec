"""In-tree builder for the serving engine's native scheduler ``dstack_amd/serving/_sched*.so``
(host C++17 + pybind11; no GPU code, so plain g++)."""

from __future__ import annotations

import subprocess
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent


def so_path() -> Path:
    return HERE / ("_sched" + sysconfig.get_config_var("EXT_SUFFIX"))


LAST = {"action": None}  # "compiled" | "reused" by the last build() call (reported by __graft_entry__)


def build(force: bool = False) -> Path:
    import pybind11

    src = HERE / "csrc" / "scheduler.cpp"
    so = so_path()
    if not force and so.exists() and so.stat().st_mtime >= src.stat().st_mtime:
        LAST["action"] = "reused"
        return so
    LAST["action"] = "compiled"
    cmd = ["g++", "-O2", "-g", "-std=c++17", "-shared", "-fPIC", "-Wall", "-Wextra",
           f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}", str(src), "-o", str(so)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"scheduler build failed:\n{r.stdout}\n{r.stderr}")
    return so


if __name__ == "__main__":
    print(build(force=True))
