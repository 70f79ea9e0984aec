"""End-to-end on CPU: real server subprocess + local backend (native ``dstack-shim`` process driver
+ ``dstack-runner``) driven through the public API and the ``dstack`` CLI (reference analogue:
the manual ``dstack apply`` flow of SURVEY §3.2; the reference has no automated e2e test)."""

import os
import subprocess
import sys
import textwrap
import time

import httpx
import pytest

from dstack_amd.native_bin import runner_path, shim_path

pytestmark = pytest.mark.skipif(not (shim_path() and runner_path()), reason="native agents not built")

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def server():
    from dstack_amd.server.testing import ServerProcess

    srv = ServerProcess().start()
    yield srv
    srv.stop()


@pytest.fixture
def client(server):
    return server.client()


def _logs(run) -> str:
    return b"".join(run.logs()).decode(errors="replace")


def _wait(run, timeout: float) -> str:
    """``run.wait`` that, on a timeout, fails with every job's status and timings."""
    try:
        return run.wait(timeout=timeout).value
    except TimeoutError as e:
        jobs = [(j.job_spec.job_num, s.status.value, s.timings) for j in run.model.jobs for s in j.job_submissions]
        pytest.fail(f"{e}; jobs: {jobs}")


def test_task_runs_and_streams_logs(client):
    from dstack_amd.api import Task

    run = client.runs.submit(Task(commands=["echo hello-$DSTACK_RUN_NAME", "echo rank=$DSTACK_NODE_RANK"],
                                  name="e2e-hello"))
    assert run.wait(timeout=180).value == "done"
    out = _logs(run)
    assert "hello-e2e-hello" in out and "rank=0" in out
    sub = run.model.jobs[0].job_submissions[-1]
    assert sub.exit_status == 0
    t = sub.timings
    assert t["submitted"] <= t["running"] <= t["first_log"] + 1e-3
    assert t["first_log"] - t["submitted"] < 10.0


def test_task_failure_exit_code(client):
    from dstack_amd.api import Task

    run = client.runs.submit(Task(commands=["echo about-to-fail", "exit 7"], name="e2e-fail"))
    assert run.wait(timeout=180).value == "failed"
    sub = run.model.jobs[0].job_submissions[-1]
    assert sub.exit_status == 7
    assert sub.termination_reason.value == "container_exited_with_error"
    assert "about-to-fail" in _logs(run)


def test_env_and_secrets_interpolation(client, server):
    from dstack_amd.api import Task

    client.api.secrets.create_or_update("main", "MY_SECRET", "s3cr3t-value")
    run = client.runs.submit(Task(commands=["echo A=$A S=$S"], env={"A": "1", "S": "${{ secrets.MY_SECRET }}"},
                                  name="e2e-env"))
    assert run.wait(timeout=180).value == "done"
    assert "A=1 S=s3cr3t-value" in _logs(run)


_FAKE_ROCPROF = r"""#!/bin/sh
# stands in for rocprofv3: records the --pmc set and the program it was put in front of, writes the
# two CSVs the runner summarises (one pair per process, -o job_%pid%), then execs the program
dir=""; pmc=""; out="job"
while [ $# -gt 0 ]; do
  case "$1" in
    -d) dir="$2"; shift 2;;
    -o) out="$2"; shift 2;;
    --pmc) shift; while [ $# -gt 0 ] && [ "${1#-}" = "$1" ]; do pmc="$pmc $1"; shift; done;;
    --) shift; break;;
    *) shift;;
  esac
done
echo "fake-rocprof pmc:$pmc"
echo "fake-rocprof program: $1 rank=${RANK:-none}"
base="$dir/$(echo "$out" | sed "s/%pid%/$$/")"
printf '"Name","Calls","TotalDurationNs"\n"gemm_kernel(float*, int)",10,5000\n' > "${base}_kernel_stats.csv"
printf 'Dispatch_Id,Kernel_Name,Counter_Name,Counter_Value\n1,"gemm_kernel(float*, int)",SQ_WAVES,64\n2,"gemm_kernel(float*, int)",SQ_WAVES,64\n1,"gemm_kernel(float*, int)",GRBM_GUI_ACTIVE,1000\n3,"norm(float*)",SQ_WAVES,8\n' > "${base}_counter_collection.csv"
exec "$@"
"""

# stands in for torchrun: --no-python runs the trailing argv once per local rank (RANK set)
_FAKE_TORCHRUN = r"""#!/bin/sh
n=1; nopy=0
while [ $# -gt 0 ]; do
  case "$1" in
    --nproc-per-node) n="$2"; shift 2;;
    --nproc-per-node=*) n="${1#*=}"; shift;;
    --no-python) nopy=1; shift;;
    -*) shift;;
    *) break;;
  esac
done
[ "$nopy" = 1 ] || { echo "fake-torchrun: rank program not wrapped"; exit 3; }
i=0
while [ $i -lt $n ]; do RANK=$i "$@" || exit $?; i=$((i + 1)); done
"""


def _fake_bin(tmp_path):
    bin_dir = tmp_path / "bin"
    bin_dir.mkdir()
    for name, text in (("rocprofv3", _FAKE_ROCPROF), ("torchrun", _FAKE_TORCHRUN)):
        f = bin_dir / name
        f.write_text(text)
        f.chmod(0o755)
    return f"{bin_dir}:{os.environ.get('PATH', '/usr/bin:/bin')}"


def test_rocprof_counters_in_job_log(client, tmp_path):
    """DSTACK_ROCPROF_COUNTERS: the runner checks the set against rocprofv3's one-pass budget, puts
    rocprofv3 directly in front of the job's program (the shell execs it; never ``-- bash -c``),
    adds ``--pmc`` and appends per-kernel sums to the job log; an over-budget set is refused with a
    log line and the job still runs (kernel statistics only)."""
    from dstack_amd.api import Task

    path = _fake_bin(tmp_path)
    run = client.runs.submit(Task(commands=["echo setup-ran", "echo job-ran"], name="e2e-rocprof",
                                  env={"PATH": path, "DSTACK_ROCPROF_COUNTERS": "SQ_WAVES,GRBM_GUI_ACTIVE"}))
    assert run.wait(timeout=180).value == "done"
    out = _logs(run)
    assert "fake-rocprof pmc: SQ_WAVES GRBM_GUI_ACTIVE" in out and "job-ran" in out and "setup-ran" in out
    assert "fake-rocprof program: echo rank=none" in out  # the program itself, not /bin/bash
    assert out.count("fake-rocprof program:") == 1  # only the last command runs under the profiler
    assert "rocprofv3 kernel statistics (1 process" in out and "gemm_kernel(float*, int) | 10 |" in out
    assert "rocprofv3 counters per kernel" in out
    assert "gemm_kernel | 2 | 128 | 1000" in out and "norm | 1 | 8 | 0" in out
    too_many = ",".join(f"SQ_C{i}" for i in range(9))
    run = client.runs.submit(Task(commands=["echo job-ran"], name="e2e-rocprof-bad",
                                  env={"PATH": path, "DSTACK_ROCPROF_COUNTERS": too_many}))
    assert run.wait(timeout=180).value == "done"
    out = _logs(run)
    assert "DSTACK_ROCPROF_COUNTERS ignored: SQ block needs 9 counters" in out
    assert "fake-rocprof pmc:\n" in out.replace("\r", "") and "job-ran" in out


def test_rocprof_per_rank_under_torchrun_and_refusal(client, tmp_path):
    """A torchrun job is profiled per rank (``torchrun --no-python rocprofv3 ... -- python3 -u
    script``; the launcher is never under the profiler) and the summaries add up over the ranks'
    CSVs; a job whose last command is a wrapper (``timeout``) is refused and runs unprofiled."""
    from dstack_amd.api import Task

    path = _fake_bin(tmp_path)
    (tmp_path / "t.py").write_text("import os; print('rank-ran', os.environ.get('RANK'))\n")
    run = client.runs.submit(Task(commands=[f"cd {tmp_path}", "torchrun --nproc-per-node=2 t.py"],
                                  name="e2e-rocprof-torchrun", env={"PATH": path, "DSTACK_ROCPROF": "1"}))
    assert run.wait(timeout=180).value == "done", _logs(run)
    out = _logs(run)
    assert "fake-rocprof program: python3 rank=0" in out and "fake-rocprof program: python3 rank=1" in out
    assert "rank-ran 0" in out and "rank-ran 1" in out
    assert "rocprofv3 kernel statistics (2 processes" in out and "gemm_kernel(float*, int) | 20 |" in out
    run = client.runs.submit(Task(commands=["timeout 30 echo wrapped-job"], name="e2e-rocprof-refused",
                                  env={"PATH": path, "DSTACK_ROCPROF": "1"}))
    assert run.wait(timeout=180).value == "done"
    out = _logs(run)
    assert "DSTACK_ROCPROF ignored: the job's last command runs 'timeout'" in out and "wrapped-job" in out
    assert "fake-rocprof" not in out


@pytest.mark.gpu
def test_rocprof_counters_on_gpu(client):
    """On the MI355X: the real rocprofv3 with --pmc, put by the runner directly in front of a tiny
    torch program (the job's shell execs it), and the per-kernel counter rows in the job log."""
    from dstack_amd.api import GPU, Resources, Task

    prog = "import torch; x = torch.ones(1 << 20, device='cuda'); print('gpu-sum', (x * 2).sum().item())"
    run = client.runs.submit(Task(commands=["echo before-profiled-step", f'python3 -c "{prog}"'],
                                  name="e2e-rocprof-gpu", resources=Resources(gpu=GPU(count=1)),
                                  env={"DSTACK_ROCPROF_COUNTERS": "SQ_WAVES,GRBM_GUI_ACTIVE"}))
    status = _wait(run, 300)
    out = _logs(run)
    print(out[-4000:])
    assert status == "done", out[-3000:]
    assert "gpu-sum 2097152.0" in out
    assert "rocprofv3 kernel statistics (1 process" in out
    assert "rocprofv3 counters per kernel" in out and "| SQ_WAVES | GRBM_GUI_ACTIVE" in out


def test_stop_long_running(client):
    from dstack_amd.api import Task

    run = client.runs.submit(Task(commands=["echo started", "sleep 300"], name="e2e-stop"))
    deadline = time.time() + 30
    while "started" not in _logs(run) and time.time() < deadline:
        time.sleep(0.2)
    run.stop(abort=False)
    st = run.wait(timeout=180)
    assert st.value in ("terminated", "aborted", "done")
    assert run.model.jobs[0].job_submissions[-1].termination_reason.value in (
        "terminated_by_user", "aborted_by_user")


def test_local_repo_code_upload(client, tmp_path):
    from dstack_amd.api import Task
    from dstack_amd.core.models.repos import LocalRepo

    (tmp_path / "train.py").write_text("print('training-script-ran', 6 * 7)\n")
    (tmp_path / ".gitignore").write_text("ignored.txt\n")
    (tmp_path / "ignored.txt").write_text("nope")
    run = client.runs.submit(Task(commands=["python3 train.py", "ls"], name="e2e-repo"), repo=LocalRepo(str(tmp_path)))
    assert run.wait(timeout=180).value == "done"
    out = _logs(run)
    assert "training-script-ran 42" in out
    assert "ignored.txt" not in out


def test_service_through_in_server_proxy(client, server):
    from dstack_amd.api import Service

    port = 18000 + os.getpid() % 1000
    conf = Service(commands=[f"python3 -m http.server {port}"], port=port, name="e2e-svc", auth=False)
    run = client.runs.submit(conf)
    url = f"{server.url}/proxy/services/main/e2e-svc/"
    deadline = time.time() + 60
    body = None
    while time.time() < deadline:
        try:
            r = httpx.get(url, timeout=2)
            if r.status_code == 200:
                body = r.text
                break
        except httpx.HTTPError:
            pass
        time.sleep(0.3)
    run.stop(abort=True)
    run.wait(timeout=180)
    assert body is not None and "Directory listing" in body


def test_llm_service_through_model_proxy(client, server):
    """A ``type: service`` replica running the serving engine (tiny random Llama on the CPU) behind
    the in-server OpenAI model proxy: chat completion request -> proxy -> replica -> engine."""
    from dstack_amd.api import Service
    from dstack_amd.core.models.services import OpenAIChatModel

    port = 19000 + os.getpid() % 1000
    cmd = (f"{sys.executable} -m dstack_amd.serving --model llama-tiny --served-model-name tiny-llama "
           f"--max-model-len 256 --max-batch 4 --port {port} --host 127.0.0.1")
    conf = Service(commands=[f"cd {REPO} && {cmd}"], port=port, name="e2e-llm", auth=False,
                   model=OpenAIChatModel(name="tiny-llama", format="openai"))
    run = client.runs.submit(conf)
    url = f"{server.url}/proxy/models/main/chat/completions"
    body = None
    deadline = time.time() + 120
    try:
        while time.time() < deadline:
            try:
                r = httpx.post(url, json={"model": "tiny-llama", "max_tokens": 4, "temperature": 0,
                                          "messages": [{"role": "user", "content": "hello"}]},
                               headers={"Authorization": f"Bearer {server.token}"}, timeout=10)
                if r.status_code == 200:
                    body = r.json()
                    break
            except httpx.HTTPError:
                pass
            time.sleep(0.5)
    finally:
        run.stop(abort=True)
        run.wait(timeout=180)
    assert body is not None, _logs(run)[-2000:]
    assert body["choices"][0]["message"]["role"] == "assistant"
    assert 1 <= body["usage"]["completion_tokens"] <= 4


def test_multinode_task_rendezvous_env(client):
    from dstack_amd.api import Task

    cmd = "echo node=$DSTACK_NODE_RANK/$DSTACK_NODES_NUM master=$DSTACK_MASTER_NODE_IP world=$WORLD_SIZE"
    run = client.runs.submit(Task(commands=[cmd], nodes=2, name="e2e-multinode"))
    assert _wait(run, 90) == "done"
    outs = sorted(b"".join(run.logs(job_num=j)).decode() for j in (0, 1))
    assert any("node=0/2" in o for o in outs) and any("node=1/2" in o for o in outs)
    assert all("master=" in o and "master= " not in o for o in outs)


def test_cli_apply_ps_logs(server, tmp_path):
    (tmp_path / ".dstack.yml").write_text(textwrap.dedent("""
        type: task
        name: e2e-cli
        commands:
          - echo cli-says-$DSTACK_RUN_NAME
          - cat data.txt
        """))
    (tmp_path / "data.txt").write_text("uploaded-data\n")
    env = dict(os.environ, DSTACK_SERVER_URL=server.url, DSTACK_TOKEN=server.token,
               DSTACK_DIR=str(tmp_path / "home"), PYTHONPATH=REPO)
    dstack = [sys.executable, "-m", "dstack_amd"]
    r = subprocess.run(dstack + ["apply", "-y"], cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "cli-says-e2e-cli" in r.stdout and "uploaded-data" in r.stdout
    r = subprocess.run(dstack + ["ps", "-a"], cwd=tmp_path, env=env, capture_output=True, text=True, timeout=180)
    assert "e2e-cli" in r.stdout
    r = subprocess.run(dstack + ["logs", "e2e-cli"], cwd=tmp_path, env=env, capture_output=True, text=True,
                       timeout=180)
    assert "uploaded-data" in r.stdout
    (tmp_path / "fail.dstack.yml").write_text("type: task\nname: e2e-cli-fail\ncommands: [\"exit 5\"]\n")
    r = subprocess.run(dstack + ["apply", "-y", "-f", "fail.dstack.yml"], cwd=tmp_path, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 5, r.stdout + r.stderr


def test_cli_offer(server, tmp_path):
    """``dstack offer``: every configured backend's offers for a spec (the local backend here)."""
    import json as _json

    env = dict(os.environ, DSTACK_SERVER_URL=server.url, DSTACK_TOKEN=server.token,
               DSTACK_DIR=str(tmp_path / "home"), PYTHONPATH=REPO)
    dstack = [sys.executable, "-m", "dstack_amd"]
    r = subprocess.run(dstack + ["offer", "--json", "-n", "5"], cwd=tmp_path, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    d = _json.loads(r.stdout)
    assert d["total_offers"] >= 1 and d["offers"][0]["backend"] == "local"
    r = subprocess.run(dstack + ["offer", "--cpu", "1..", "--on-demand"], cwd=tmp_path, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "BACKEND" in r.stdout and "offers shown" in r.stdout, r.stdout + r.stderr
    r = subprocess.run(dstack + ["offer", "--gpu", "MI355X:1024"], cwd=tmp_path, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and "0 of 0 offers shown" in r.stdout, r.stdout + r.stderr


def test_service_through_local_gateway(tmp_path):
    """Gateway on the server host (built-in data plane): service registered on the gateway,
    replica upstream registered when the job runs, Host-routed request reaches the replica."""
    from dstack_amd.api import Service
    from dstack_amd.core.models.gateways import GatewayConfiguration
    from dstack_amd.server.testing import ServerProcess, free_port

    with ServerProcess() as srv:
        c = srv.client()
        gw = c.api.gateways.create("main", GatewayConfiguration(name="gw", backend="local", region="local",
                                                                domain="apps.test", default=True))
        deadline = time.time() + 30
        while gw.status.value != "running" and time.time() < deadline:
            time.sleep(0.2)
            gw = c.api.gateways.get("main", "gw")
        assert gw.status.value == "running", gw.status_message
        port = free_port()
        run = c.runs.submit(Service(commands=[f"python3 -m http.server {port}"], port=port, name="gwsvc", https=False,
                                    auth=False))
        assert run.model.service.url == "http://gwsvc.apps.test"
        data_plane = f"http://{gw.hostname}/"
        body = None
        deadline = time.time() + 60
        while time.time() < deadline:
            try:
                r = httpx.get(data_plane, headers={"host": "gwsvc.apps.test"}, timeout=2)
                if r.status_code == 200:
                    body = r.text
                    break
            except httpx.HTTPError:
                pass
            time.sleep(0.3)
        run.stop(abort=True)
        run.wait(timeout=180)
        c.api.gateways.delete("main", ["gw"])
        assert body is not None and "Directory listing" in body


@pytest.mark.timeout(1600)  # a sanitizer build from scratch beside a loaded parallel run
@pytest.mark.parametrize("target", ["test", "test-tsan", "test-asan"])
def test_native_unit_tests(target):
    """C++ unit tests of the agents (JSON, log history, xGMI placement, GPU lock, HTTP), plain and
    under ThreadSanitizer / AddressSanitizer+UBSan (host code; the Go reference runs -race)."""
    r = subprocess.run(["make", "-C", os.path.join(REPO, "native"), target], capture_output=True, text=True,
                       timeout=1500)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]


class _LocalPool:
    """Stands in for the SSH TunnelPool: runs the deploy commands on this host under a temp HOME."""

    def __init__(self, home):
        self.home = home

    def run(self, target, private_key, command, timeout=600, input=None):
        env = dict(os.environ, HOME=str(self.home))
        return subprocess.run(["bash", "-c", command], env=env, input=input, capture_output=True, timeout=timeout)

    def copy(self, target, private_key, local_path, remote_path, timeout=600):
        import shutil

        dst = os.path.join(self.home, remote_path)
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        shutil.copy(local_path, dst)
        return subprocess.CompletedProcess([], 0, b"", b"")


def test_ssh_fleet_deploy_flow(tmp_path, monkeypatch):
    """deploy_ssh_instance end to end minus the ssh transport: agents copied, shim.env written,
    shim started (pid file), host_info read back and turned into an instance type."""
    import signal

    from dstack_amd.core.backends import remote
    from dstack_amd.core.models.instances import RemoteConnectionInfo, SSHKey
    from dstack_amd.server.testing import free_port

    home = tmp_path / "home"
    home.mkdir()
    monkeypatch.setattr(remote, "get_tunnel_pool", lambda: _LocalPool(home))
    port = free_port()
    rci = RemoteConnectionInfo(host="10.0.0.5", port=22, ssh_user="ubuntu",
                               ssh_keys=[SSHKey(public="ssh-ed25519 AAAA k")],
                               env={"DSTACK_SHIM_HTTP_PORT": str(port)})
    try:
        info = remote.deploy_ssh_instance(rci, "ssh-ed25519 AAAA project", "unused-private-key", timeout=60)
        shim_dir = home / ".dstack-shim"
        assert (shim_dir / "dstack-shim").exists() and (shim_dir / "dstack-runner").exists()
        assert f"DSTACK_SHIM_HTTP_PORT={port}" in (shim_dir / "shim.env").read_text()
        assert "ssh-ed25519 AAAA project" in (home / ".ssh" / "authorized_keys").read_text()
        itype, topo = remote.host_info_to_instance_type(info)
        assert itype.resources.cpus >= 1 and itype.resources.memory_mib > 0
        r = httpx.get(f"http://127.0.0.1:{port}/api/healthcheck", timeout=5)
        assert r.json()["service"] == "dstack-shim"
    finally:
        pid_file = home / ".dstack-shim" / "shim.pid"
        if pid_file.exists():
            try:
                os.kill(int(pid_file.read_text().strip()), signal.SIGTERM)
            except (ProcessLookupError, ValueError):
                pass


def test_cli_deprecated_run_and_pool(server, tmp_path):
    """``dstack run DIR`` (deprecated alias of apply) and the ``dstack pool`` subcommands."""
    proj = tmp_path / "proj"
    proj.mkdir()
    (proj / ".dstack.yml").write_text("type: task\nname: e2e-run\ncommands: [\"echo via-run\"]\n")
    env = dict(os.environ, DSTACK_SERVER_URL=server.url, DSTACK_TOKEN=server.token,
               DSTACK_DIR=str(tmp_path / "home"), PYTHONPATH=REPO)
    dstack = [sys.executable, "-m", "dstack_amd"]
    r = subprocess.run(dstack + ["run", str(proj), "-y"], cwd=tmp_path, env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    if "via-run" not in r.stdout:  # tell a lost log line from a CLI streaming race
        stored = subprocess.run(dstack + ["logs", "e2e-run"], cwd=tmp_path, env=env, capture_output=True, text=True,
                                timeout=60)
        diag = subprocess.run(dstack + ["logs", "e2e-run", "-d"], cwd=tmp_path, env=env, capture_output=True,
                              text=True, timeout=60)
        pytest.fail(f"apply output lacks the job's line; stored logs: {stored.stdout!r}; runner log tail: "
                    f"{diag.stdout[-1500:]!r}")
    assert "deprecated" in r.stdout
    r = subprocess.run(dstack + ["pool", "create", "-n", "cli-pool"], env=env, capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    r = subprocess.run(dstack + ["pool", "list"], env=env, capture_output=True, text=True, timeout=60)
    assert "cli-pool" in r.stdout, r.stdout + r.stderr
    key = tmp_path / "id_test"
    key.write_text("-----BEGIN OPENSSH PRIVATE KEY-----\nx\n-----END OPENSSH PRIVATE KEY-----\n")
    (tmp_path / "id_test.pub").write_text("ssh-ed25519 AAAATEST test\n")
    r = subprocess.run(dstack + ["pool", "add-ssh", "ubuntu@192.0.2.10", "-i", str(key), "--pool", "cli-pool",
                                 "--name", "onprem-0"], env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    r = subprocess.run(dstack + ["pool", "ps", "--pool", "cli-pool"], env=env, capture_output=True, text=True,
                       timeout=60)
    assert "onprem-0" in r.stdout, r.stdout + r.stderr
    r = subprocess.run(dstack + ["pool", "rm", "onprem-0", "--pool", "cli-pool", "-y", "--force"], env=env,
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
