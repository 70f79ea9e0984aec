"""The torch-free per-GPU launcher (dstack_amd/workloads/launch.py): torchrun-compatible rank
environment, failure propagation, signal forwarding, and that it never imports torch."""

import os
import signal
import subprocess
import sys
import time

from dstack_amd.workloads import launch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rank_env_matches_torchrun_layout():
    envs = launch.build_rank_envs(nnodes=2, node_rank=1, nproc=4, master_addr="10.0.0.1", master_port=29600, base={})
    assert [e["RANK"] for e in envs] == ["4", "5", "6", "7"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert {e["WORLD_SIZE"] for e in envs} == {"8"} and {e["LOCAL_WORLD_SIZE"] for e in envs} == {"4"}
    assert {e["GROUP_RANK"] for e in envs} == {"1"} and {e["MASTER_ADDR"] for e in envs} == {"10.0.0.1"}
    assert {e["MASTER_PORT"] for e in envs} == {"29600"}


def _run(args, tmp_path, timeout=60, **kw):
    env = dict(os.environ, PYTHONPATH=REPO)
    return subprocess.run([sys.executable, "-m", "dstack_amd.workloads.launch", *args], cwd=tmp_path, env=env,
                          capture_output=True, text=True, timeout=timeout, **kw)


def test_ranks_run_and_torch_is_not_imported_by_the_launcher(tmp_path):
    (tmp_path / "rank.py").write_text(
        "import os, sys\n"
        "print('rank', os.environ['RANK'], os.environ['LOCAL_RANK'], os.environ['WORLD_SIZE'], sys.argv[1:])\n")
    r = _run(["--nnodes=1", "--nproc-per-node", "3", "--master-port=29777", "rank.py", "--x", "1"], tmp_path)
    assert r.returncode == 0, r.stderr
    lines = sorted(ln for ln in r.stdout.splitlines() if ln.startswith("rank"))
    assert lines == [f"rank {i} {i} 3 ['--x', '1']" for i in range(3)]
    probe = subprocess.run([sys.executable, "-c", "import sys; import dstack_amd.workloads.launch; "
                            "print('torch' in sys.modules)"], env=dict(os.environ, PYTHONPATH=REPO),
                           capture_output=True, text=True, timeout=60)
    assert probe.stdout.strip() == "False"


def test_a_failing_rank_stops_its_siblings_with_its_exit_code(tmp_path):
    (tmp_path / "rank.py").write_text(
        "import os, sys, time\n"
        "if os.environ['LOCAL_RANK'] == '1':\n    time.sleep(0.3); sys.exit(3)\n"
        "time.sleep(60)\n")
    t0 = time.time()
    r = _run(["--nproc-per-node", "3", "rank.py"], tmp_path)
    assert r.returncode == 3 and time.time() - t0 < 30


def test_sigterm_is_forwarded_to_every_rank(tmp_path):
    (tmp_path / "rank.py").write_text(
        "import os, signal, sys, time\n"
        "def h(*a):\n    open(f\"term{os.environ['LOCAL_RANK']}\", 'w').close(); sys.exit(0)\n"
        "signal.signal(signal.SIGTERM, h)\nopen(f\"up{os.environ['LOCAL_RANK']}\", 'w').close()\ntime.sleep(60)\n")
    p = subprocess.Popen([sys.executable, "-m", "dstack_amd.workloads.launch", "--nproc-per-node", "2", "rank.py"],
                         cwd=tmp_path, env=dict(os.environ, PYTHONPATH=REPO))
    deadline = time.time() + 30
    while not ((tmp_path / "up0").exists() and (tmp_path / "up1").exists()) and time.time() < deadline:
        time.sleep(0.05)
    p.send_signal(signal.SIGTERM)
    rc = p.wait(timeout=30)
    assert (tmp_path / "term0").exists() and (tmp_path / "term1").exists()
    assert rc == 128 + signal.SIGTERM


def test_no_python_runs_the_program_directly(tmp_path):
    r = _run(["--nproc-per-node", "2", "--no-python", "/bin/sh", "-c", "echo r$RANK"], tmp_path)
    assert r.returncode == 0 and sorted(r.stdout.split()) == ["r0", "r1"]
