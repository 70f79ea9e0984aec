"""One process per GPU, without importing torch in the launcher.

``python -m dstack_amd.workloads.launch [--nnodes N] [--node-rank R] [--nproc-per-node G]
[--master-addr A] [--master-port P] [--no-python] script.py [args...]``

The options are torchrun's (the subset a static, non-elastic job uses), so a task's ``torchrun``
line can switch launchers by name, and the runner's per-rank profiling (``DSTACK_ROCPROF``,
native/runner/rocprof.cpp) treats it like torchrun (``--no-python rocprofv3 ... -- python -u``).

Why: torchrun imports torch (~1.5 s on MI355X hosts) before it spawns ranks that import it again,
and that import sits on the critical path of every job's start (bench_apply.py stage
``launch_s``).  This launcher only sets the ``env://`` rendezvous variables torch.distributed reads
(RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, GROUP_RANK, MASTER_ADDR, MASTER_PORT) and starts
the ranks; the dstack runner already provides the cluster facts (``DSTACK_NODES_NUM`` ...).
Failure handling: the first rank that exits non-zero terminates its siblings (SIGTERM, SIGKILL
after a grace period) and its exit code becomes the launcher's; SIGTERM/SIGINT to the launcher is
forwarded to every rank.  No restarts (a failed job is retried by the run's retry policy).
"""

from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import time
from typing import List, Optional

GRACE_S = 10.0


def build_rank_envs(nnodes: int, node_rank: int, nproc: int, master_addr: str, master_port: int,
                    base: Optional[dict] = None) -> List[dict]:
    base = dict(os.environ if base is None else base)
    world = nnodes * nproc
    envs = []
    for lr in range(nproc):
        e = dict(base)
        e.update(RANK=str(node_rank * nproc + lr), LOCAL_RANK=str(lr), WORLD_SIZE=str(world),
                 LOCAL_WORLD_SIZE=str(nproc), GROUP_RANK=str(node_rank), GROUP_WORLD_SIZE=str(nnodes),
                 ROLE_RANK=str(node_rank * nproc + lr), ROLE_WORLD_SIZE=str(world),
                 MASTER_ADDR=master_addr, MASTER_PORT=str(master_port), TORCHELASTIC_RESTART_COUNT="0")
        envs.append(e)
    return envs


def parse(argv: List[str]):
    ap = argparse.ArgumentParser(prog="python -m dstack_amd.workloads.launch", allow_abbrev=False)
    for opt, typ, default in (("nnodes", int, 1), ("node-rank", int, 0), ("nproc-per-node", int, 1),
                              ("master-addr", str, "127.0.0.1"), ("master-port", int, 29500)):
        ap.add_argument(f"--{opt}", f"--{opt.replace('-', '_')}", type=typ, default=default)
    ap.add_argument("--no-python", "--no_python", action="store_true",
                    help="run the program directly instead of `python -u program`")
    ap.add_argument("program")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    return ap.parse_args(argv)


def main(argv: Optional[List[str]] = None) -> int:
    a = parse(sys.argv[1:] if argv is None else argv)
    if a.nproc_per_node < 1 or a.nnodes < 1 or not 0 <= a.node_rank < a.nnodes:
        print(f"launch: bad layout nnodes={a.nnodes} node_rank={a.node_rank} nproc={a.nproc_per_node}",
              file=sys.stderr)
        return 2
    cmd = [a.program, *a.args] if a.no_python else [sys.executable, "-u", a.program, *a.args]
    procs = [subprocess.Popen(cmd, env=e) for e in
             build_rank_envs(a.nnodes, a.node_rank, a.nproc_per_node, a.master_addr, a.master_port)]
    stopping = {"sig": None}

    def _forward(signum, _frame):
        stopping["sig"] = signum
        for p in procs:
            if p.poll() is None:
                p.send_signal(signum)

    signal.signal(signal.SIGTERM, _forward)
    signal.signal(signal.SIGINT, _forward)
    rc = 0
    while True:
        alive = [p for p in procs if p.poll() is None]
        failed = [p for p in procs if p.returncode not in (None, 0)]
        if failed and rc == 0:
            rc = failed[0].returncode if failed[0].returncode > 0 else 128 - failed[0].returncode
            for p in alive:  # one rank failed: the collective job cannot finish, stop the rest
                p.terminate()
            deadline = time.time() + GRACE_S
            while any(p.poll() is None for p in procs) and time.time() < deadline:
                time.sleep(0.05)
            for p in procs:
                if p.poll() is None:
                    p.kill()
        if not alive:
            break
        time.sleep(0.05)
    if stopping["sig"] is not None and rc == 0:
        rc = 128 + stopping["sig"]
    return rc


if __name__ == "__main__":
    sys.exit(main())
