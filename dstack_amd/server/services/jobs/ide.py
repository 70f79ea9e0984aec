"""IDE bootstrap for ``type: dev-environment`` (reference:
``S/services/jobs/configurators/extensions/vscode.py:15-45`` and ``configurators/dev.py``).

``ide: vscode`` with ``version: <commit>`` pre-installs the VS Code Server of exactly that commit
(the one the user's desktop VS Code runs, so Remote-SSH attaches without downloading anything) plus
the Python and Jupyter extensions, then prints the ``vscode://`` link.  Without ``version`` the
desktop installs the server itself on first connect.  The commands run in the job's shell before
the user's ``init`` and work with either curl or wget (ROCm images ship one or the other).
"""

from __future__ import annotations

import re
import shlex
from typing import List, Optional

DEFAULT_EXTENSIONS = ("ms-python.python", "ms-toolsai.jupyter")

INSTALL_IPYKERNEL = ("(echo 'pip install ipykernel...' && pip install -q --no-cache-dir ipykernel 2>/dev/null) || "
                     "echo 'no pip, ipykernel was not installed'")

_COMMIT = re.compile(r"^[0-9a-f]{7,40}$")


class VSCodeServer:
    def __init__(self, run_name: str, version: Optional[str], extensions=DEFAULT_EXTENSIONS,
                 workdir: str = "/workflow"):
        if version is not None and not _COMMIT.match(version):
            raise ValueError(f"vscode version must be a commit hash (Help > About in VS Code), got {version!r}")
        self.run_name = run_name
        self.version = version
        self.extensions = list(extensions)
        self.workdir = workdir

    def install_commands(self) -> List[str]:
        if self.version is None:
            return []
        target = f'"$HOME/.vscode-server/bin/{self.version}"'
        url = f"https://update.code.visualstudio.com/commit:{self.version}/server-linux-$arch/stable"
        archive = '"/tmp/vscode-server-$arch.tar.gz"'
        cmds = [
            'case "$(uname -m)" in aarch64|arm64) arch=arm64 ;; *) arch=x64 ;; esac',
            f"mkdir -p /tmp {target}",
            f'(command -v curl >/dev/null && curl -fsSL "{url}" -o {archive}) || wget -q "{url}" -O {archive}',
            f"tar --no-same-owner -xz --strip-components=1 -C {target} -f {archive}",
            f"rm -f {archive}",
        ]
        if self.extensions:
            exts = " ".join(f"--install-extension {shlex.quote(e)}" for e in self.extensions)
            cmds.append(f'PATH="$PATH:{target[1:-1]}/bin" code-server {exts}')
        return cmds

    def link(self) -> str:
        return f"vscode://vscode-remote/ssh-remote+{self.run_name}{self.workdir}"

    def readme_commands(self) -> List[str]:
        return [
            "echo 'To open in VS Code Desktop, use link below:'",
            "echo ''",
            f"echo '  {self.link()}'",
            "echo ''",
            f"echo 'To connect via SSH, use: `ssh {self.run_name}`'",
            "echo ''",
            "echo -n 'To exit, press Ctrl+C.'",
        ]


def dev_environment_commands(conf, run_name: str) -> List[str]:
    """The shell of a dev-environment job: IDE server, ipykernel, ``setup``, ``init``, the
    connection instructions, then idle until stopped."""
    ide = VSCodeServer(run_name or "dev", conf.version, workdir=conf.working_dir or "/workflow")
    cmds = ide.install_commands()
    cmds.append(INSTALL_IPYKERNEL)
    cmds += list(conf.setup)
    cmds.append("echo ''")
    cmds += list(conf.init)
    cmds += ide.readme_commands()
    cmds.append("tail -f /dev/null")  # idle
    return cmds
