"""In-tree builder for the HIP extension ``dstack_amd/ops/_C*.so`` (gfx950 only).

Kernels (``csrc/*.hip``) are compiled by ``hipcc --offload-arch=gfx950`` as plain HIP translation
units (no torch headers, no hipify); ``csrc/bindings.cpp`` is the only torch-aware file.  Objects
are rebuilt when their sources or headers change.

    python -m dstack_amd.ops.build            # build
    python -m dstack_amd.ops.build --asm      # also keep .s (register/occupancy audit)
"""

from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
BUILD = HERE.parent.parent / "build" / "ops"
ARCH = os.environ.get("DSTACK_AMD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce

    inc = ce.include_paths(device_type="cuda")
    lib = ce.library_paths(device_type="cuda")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def so_path() -> Path:
    return HERE / ("_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def _newer(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r.stderr


def build(verbose: bool = False, keep_asm: bool = False, force: bool = False) -> Path:
    BUILD.mkdir(parents=True, exist_ok=True)
    headers = list(CSRC.glob("*.h"))
    kernels = sorted(CSRC.glob("*.hip"))
    common = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-D__HIP_PLATFORM_AMD__=1"]
    jobs = []
    objs = []
    for src in kernels:
        obj = BUILD / (src.stem + ".o")
        objs.append(obj)
        if force or _newer(obj, [src, *headers]):
            cmd = [HIPCC, *common, "-c", str(src), "-o", str(obj)]
            if keep_asm:
                cmd += ["-save-temps=obj", "-Rpass-analysis=kernel-resource-usage"]
            jobs.append(cmd)
    inc, lib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    bsrc = CSRC / "bindings.cpp"
    bobj = BUILD / "bindings.o"
    objs.append(bobj)
    if force or _newer(bobj, [bsrc]):
        jobs.append(
            [
                "g++", "-O2", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_C",
                "-DTORCH_API_INCLUDE_EXTENSION_H", *[f"-I{p}" for p in inc], f"-I{py_inc}",
                "-w", "-c", str(bsrc), "-o", str(bobj),
            ]
        )
    with cf.ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        for out in ex.map(_run, jobs):
            if verbose and out:
                print(out, file=sys.stderr)
    so = so_path()
    if force or _newer(so, objs):
        link = [
            HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(so),
            *[f"-L{p}" for p in lib], *[f"-Wl,-rpath,{p}" for p in lib],
            "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
            "-lamdhip64",
        ]
        _run(link)
    return so


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm", action="store_true")
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", action="store_true")
    a = ap.parse_args()
    print(build(verbose=a.v, keep_asm=a.asm, force=a.force))


if __name__ == "__main__":
    main()
