"""``type: dev-environment`` IDE bootstrap (reference ``configurators/extensions/vscode.py:15-45``):
the VS Code Server of the pinned commit plus the Python/Jupyter extensions are installed before
``init``, the ``vscode://`` link is printed, and the job idles.  The generated shell is executed
here against a stand-in ``curl`` that serves a fake server archive."""

import os
import subprocess
import tarfile

import pytest

from dstack_amd.core.models.runs import RunSpec
from dstack_amd.server.services.jobs.configurators import get_job_specs_from_run_spec

COMMIT = "1a5daa3a0231a0fbba4f14db7ec463cf99d7768e"


def _spec(**conf):
    return RunSpec.model_validate({"run_name": "my-dev", "repo_id": "r", "repo_data": {"repo_type": "virtual"},
                                   "configuration": {"type": "dev-environment", "ide": "vscode",
                                                     "image": "rocm/pytorch:latest", **conf}})


def test_pinned_version_installs_server_extensions_and_prints_link():
    js = get_job_specs_from_run_spec(_spec(version=COMMIT, init=["echo init-done"], setup=["echo setup-done"]))[0]
    assert js.commands[:2] == ["/bin/bash", "-c"]
    script = js.commands[2]
    assert f"commit:{COMMIT}/server-linux-$arch/stable" in script
    assert "--install-extension ms-python.python --install-extension ms-toolsai.jupyter" in script
    assert "vscode://vscode-remote/ssh-remote+my-dev/workflow" in script
    # order: server install, ipykernel, setup, init, readme, idle
    idx = [script.index(x) for x in ("tar --no-same-owner", "ipykernel", "setup-done", "init-done", "vscode://",
                                     "tail -f /dev/null")]
    assert idx == sorted(idx)
    assert js.max_duration == 6 * 3600  # dev environments stop after 6 h by default


def test_without_version_no_server_download():
    script = get_job_specs_from_run_spec(_spec())[0].commands[2]
    assert "update.code.visualstudio.com" not in script and "vscode://" in script


def test_version_must_be_a_commit():
    with pytest.raises(Exception, match="commit"):
        _spec(version="1.85.2")


def test_install_commands_run(tmp_path):
    """Run the generated install steps with a fake curl serving an archive whose code-server records
    the extensions it was asked to install."""
    pkg = tmp_path / "pkg"
    (pkg / "vscode-server-linux-x64" / "bin").mkdir(parents=True)
    cs = pkg / "vscode-server-linux-x64" / "bin" / "code-server"
    cs.write_text(f"#!/bin/sh\necho \"$@\" > {tmp_path}/installed\n")
    cs.chmod(0o755)
    archive = tmp_path / "server.tar.gz"
    with tarfile.open(archive, "w:gz") as t:
        t.add(pkg / "vscode-server-linux-x64", arcname="vscode-server-linux-x64")
    bindir = tmp_path / "bin"
    bindir.mkdir()
    (bindir / "curl").write_text(f"#!/bin/sh\nwhile [ $# -gt 0 ]; do [ \"$1\" = -o ] && cp {archive} \"$2\"; "
                                 "shift; done\n")
    (bindir / "curl").chmod(0o755)
    from dstack_amd.server.services.jobs.ide import VSCodeServer

    cmds = VSCodeServer("my-dev", COMMIT).install_commands()
    env = dict(os.environ, HOME=str(tmp_path / "home"), PATH=f"{bindir}:{os.environ['PATH']}")
    r = subprocess.run(["bash", "-c", " && ".join(cmds)], env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "home" / ".vscode-server" / "bin" / COMMIT / "bin" / "code-server").exists()
    assert (tmp_path / "installed").read_text().split() == ["--install-extension", "ms-python.python",
                                                             "--install-extension", "ms-toolsai.jupyter"]
