"""In-tree builder for the HIP extension ``dstack_amd/ops/_C*.so`` (gfx950 only).

Kernels (``csrc/*.hip``) are compiled by ``hipcc --offload-arch=gfx950`` as plain HIP translation
units (no torch headers, no hipify); ``csrc/bindings.cpp`` is the only torch-aware file.  Rebuilds
are content-addressed, not mtime-based: every object records the SHA-256 of its source, the headers
and the compile command (``<obj>.sha256``), and the extension records the hash of its objects and
the link command (``_C.sha256`` next to the ``.so``), so a copied / checked-out tree with fresh
mtimes is not rebuilt needlessly and an edited source is never missed.

    python -m dstack_amd.ops.build            # build
    python -m dstack_amd.ops.build --asm      # also keep .s (register/occupancy audit)
    python -m dstack_amd.ops.build --check    # exit 1 unless the .so matches the current sources
    python -m dstack_amd.ops.build --check-toolchain   # hipcc present and able to target gfx950
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
ROOT = HERE.parent.parent
BUILD = ROOT / "build" / "ops"
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


def _portable(cmd) -> str:
    """A command line with the repository's location factored out: the tree is built here and run
    from wherever the GPU box unpacks it, and the same sources + flags must give the same digest."""
    return "\0".join(cmd).replace(str(ROOT), "<repo>")


def _digest(files, cmd) -> str:
    import hashlib

    h = hashlib.sha256()
    for f in files:
        h.update(Path(f).name.encode() + b"\0" + Path(f).read_bytes() + b"\0")
    h.update(_portable(cmd).encode())
    return h.hexdigest()


def _stale(target: Path, digest: str) -> bool:
    stamp = target.with_name(target.name + ".sha256")
    return not target.exists() or not stamp.exists() or stamp.read_text().strip() != digest


def _stamp(target: Path, digest: str) -> None:
    target.with_name(target.name + ".sha256").write_text(digest + "\n")


def so_stamp_path() -> Path:
    return HERE / "_C.sha256"


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r.stderr


def _plan(keep_asm: bool = False):
    """[(object, compile command, digest)] and the link command."""
    headers = sorted(CSRC.glob("*.h"))
    kernels = sorted(CSRC.glob("*.hip"))
    common = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-D__HIP_PLATFORM_AMD__=1"]
    units = []
    for src in kernels:
        obj = BUILD / (src.stem + ".o")
        cmd = [HIPCC, *common, "-c", str(src), "-o", str(obj)]
        if keep_asm:
            cmd += ["-save-temps=obj", "-Rpass-analysis=kernel-resource-usage"]
        units.append((obj, cmd, _digest([src, *headers], cmd)))
    inc, lib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    bsrc = CSRC / "bindings.cpp"
    bobj = BUILD / "bindings.o"
    bcmd = [
        "g++", "-O2", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_C",
        "-DTORCH_API_INCLUDE_EXTENSION_H", *[f"-I{p}" for p in inc], f"-I{py_inc}",
        "-w", "-c", str(bsrc), "-o", str(bobj),
    ]
    units.append((bobj, bcmd, _digest([bsrc], bcmd)))
    link = [
        HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *[str(u[0]) for u in units], "-o", str(so_path()),
        *[f"-L{p}" for p in lib], *[f"-Wl,-rpath,{p}" for p in lib],
        "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python", "-lamdhip64",
    ]
    import hashlib

    so_digest = hashlib.sha256(("\0".join(u[2] for u in units) + "\0" + _portable(link)).encode()).hexdigest()
    return units, link, so_digest


def is_current() -> bool:
    """True when the built extension was linked from exactly the current sources and flags."""
    so = so_path()
    _, _, so_digest = _plan()
    stamp = so_stamp_path()
    return so.exists() and stamp.exists() and stamp.read_text().strip() == so_digest


def quick_key() -> str:
    """A digest of everything the build reads that can be had WITHOUT importing torch: the kernel
    sources and headers, the torch installation's version file and location, the Python headers'
    location, the arch and the compiler.  Equal to the manifest's -> the .so is current, and a job
    whose first command is ``python -m dstack_amd.ops.build`` does not pay a torch import (~2 s)
    to find that out."""
    import hashlib
    import importlib.util

    h = hashlib.sha256()
    for f in sorted(CSRC.glob("*.h")) + sorted(CSRC.glob("*.hip")) + [CSRC / "bindings.cpp", Path(__file__)]:
        h.update(f.name.encode() + b"\0" + f.read_bytes() + b"\0")
    spec = importlib.util.find_spec("torch")
    tdir = Path(spec.origin).parent if spec and spec.origin else None
    h.update(str(tdir).encode())
    if tdir is not None and (tdir / "version.py").exists():
        h.update((tdir / "version.py").read_bytes())
    h.update("\0".join([ARCH, HIPCC, sysconfig.get_paths()["include"], sysconfig.get_config_var("EXT_SUFFIX")]).encode())
    return h.hexdigest()


def _quick_current() -> bool:
    import hashlib
    import json

    so = so_path()
    try:
        m = json.loads(manifest_path().read_text())
        return (so.exists() and m.get("quick_key") == quick_key()
                and hashlib.sha256(so.read_bytes()).hexdigest() == m.get("so_sha256"))
    except (OSError, ValueError):
        return False


_PROBE_SRC = "#include <hip/hip_runtime.h>\n__global__ void k(float* p) { p[threadIdx.x] = 1.f; }\n"


def check_toolchain() -> str:
    """hipcc must exist and target gfx950 (ROCm >= 7.0).  Returns the HIP version line; raises a
    RuntimeError that says what is wrong and what to use instead -- the typical failure is a ROCm 6.x
    container image on an MI350X/MI355X host, whose compiler has no gfx950 target."""
    from dstack_amd.core.models.images import DEFAULT_ROCM_IMAGE

    if not Path(HIPCC).exists():
        raise RuntimeError(f"hipcc not found at {HIPCC}: the HIP kernels need ROCm >= 7.0 for {ARCH} "
                           f"(set HIPCC, or run in {DEFAULT_ROCM_IMAGE})")
    ver = subprocess.run([HIPCC, "--version"], capture_output=True, text=True).stdout
    line = next((x for x in ver.splitlines() if "HIP version" in x), "HIP version: unknown")
    import tempfile

    with tempfile.TemporaryDirectory(prefix="dsa_hipcc_") as td:  # (hipcc does not read stdin)
        src = Path(td) / "probe.hip"
        src.write_text(_PROBE_SRC)
        r = subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-c", str(src), "-o", str(Path(td) / "probe.o")],
                           capture_output=True, text=True)
    if r.returncode != 0:
        rocm = ""
        info = Path(HIPCC).resolve().parent.parent / ".info" / "version"
        if info.exists():
            rocm = f" (ROCm {info.read_text().strip()})"
        raise RuntimeError(f"{HIPCC}{rocm}, {line.strip()}: cannot compile for --offload-arch={ARCH}; "
                           f"MI350X/MI355X (gfx950) need ROCm >= 7.0 -- use {DEFAULT_ROCM_IMAGE}.\n"
                           f"{r.stderr.strip()[-600:]}")
    return line.strip()


def build(verbose: bool = False, keep_asm: bool = False, force: bool = False) -> Path:
    if not force and not keep_asm and _quick_current():
        return so_path()  # nothing changed since the recorded build (no torch import needed)
    BUILD.mkdir(parents=True, exist_ok=True)
    units, link, so_digest = _plan(keep_asm)
    jobs = [(obj, cmd, d) for obj, cmd, d in units if force or _stale(obj, d)]
    if jobs:
        check_toolchain()  # a clear message instead of a wall of clang errors
    # a unit's stamp is dropped before it compiles and written by the worker right after it succeeds:
    # when another unit fails, a unit that compiled must not keep the stamp of its PREVIOUS sources
    # (reverting those sources would then reuse the new object under the old stamp)
    for obj, _, _ in jobs:
        obj.with_name(obj.name + ".sha256").unlink(missing_ok=True)

    def compile_unit(j):
        out = _run(j[1])
        _stamp(j[0], j[2])
        return out

    with cf.ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        for out in ex.map(compile_unit, jobs):
            if verbose and out:
                print(out, file=sys.stderr)
    so = so_path()
    linked = False
    if force or jobs or not is_current():
        _run(link)
        so_stamp_path().write_text(so_digest + "\n")
        linked = True
    _write_manifest(so, so_digest, [Path(j[0]).stem for j in jobs], [Path(u[0]).stem for u in units], linked)
    return so


def manifest_path() -> Path:
    return so_path().with_name("_C.manifest.json")


def _write_manifest(so: Path, so_digest: str, compiled, units, linked: bool):
    """Build provenance next to the .so: which sources/flags it was linked from (``source_digest``),
    the binary's own hash, and what this build call compiled versus reused from the
    content-addressed cache.  ``verify_loaded`` checks it against the library a process mapped."""
    import datetime
    import hashlib
    import json
    import platform

    prev = {}
    if manifest_path().exists():
        try:
            prev = json.loads(manifest_path().read_text())
        except ValueError:
            prev = {}
    ver = subprocess.run([HIPCC, "--version"], capture_output=True, text=True).stdout.splitlines()
    m = {
        "so": so.name, "so_sha256": hashlib.sha256(so.read_bytes()).hexdigest(), "source_digest": so_digest,
        "arch": ARCH, "hipcc": next((x for x in ver if "HIP version" in x), ver[0] if ver else ""),
        "units": units, "compiled_now": compiled, "linked_now": linked,
        "built_at": datetime.datetime.now(datetime.timezone.utc).isoformat(timespec="seconds")
        if (compiled or linked or not prev) else prev.get("built_at"),
        "built_on": platform.node() if (compiled or linked or not prev) else prev.get("built_on"),
        "quick_key": quick_key(),
    }
    manifest_path().write_text(json.dumps(m, indent=1) + "\n")


def verify_loaded(loaded_so: str) -> dict:
    """Provenance of the extension a process actually loaded: its hash must equal the manifest's,
    and the manifest's source digest must equal the digest of the kernel sources in this tree --
    i.e. the running kernels were compiled from exactly these sources.  Raises otherwise."""
    import hashlib
    import json

    m = json.loads(manifest_path().read_text())
    got = hashlib.sha256(Path(loaded_so).read_bytes()).hexdigest()
    if got != m["so_sha256"]:
        raise RuntimeError(f"{loaded_so}: binary differs from the build manifest ({got[:12]} vs {m['so_sha256'][:12]})")
    _, _, digest = _plan()
    if m["source_digest"] != digest:
        raise RuntimeError(f"{loaded_so} was built from other kernel sources than this tree's: rebuild")
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm", action="store_true")
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", action="store_true")
    ap.add_argument("--check", action="store_true", help="exit 1 unless the .so matches the current sources")
    ap.add_argument("--check-toolchain", action="store_true", help="only check that hipcc targets gfx950")
    a = ap.parse_args()
    if a.check_toolchain:
        try:
            print(f"{HIPCC}: {check_toolchain()}, --offload-arch={ARCH} ok")
        except RuntimeError as e:
            print(f"error: {e}", file=sys.stderr)
            sys.exit(1)
        return
    if a.check:
        ok = is_current()
        print(f"{so_path()}: {'current' if ok else 'STALE or missing'}")
        sys.exit(0 if ok else 1)
    try:
        print(build(verbose=a.v, keep_asm=a.asm, force=a.force))
    except RuntimeError as e:
        print(f"error: {e}", file=sys.stderr)
        sys.exit(1)


if __name__ == "__main__":
    main()
