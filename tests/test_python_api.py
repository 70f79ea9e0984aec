"""The public Python API (``dstack_amd.api``: ``Client`` and its collections, reference
``src/dstack/api/_public/*``) against the in-process server: backends, fleets, volumes, runs
(plan, submit, list, get, stop) and the users/projects endpoints of ``APIClient``."""

from __future__ import annotations

import pytest

from dstack_amd.api import APIClient, Client, GPU, Resources, Task, VirtualRepo
from dstack_amd.core.errors import ServerClientError


@pytest.fixture
def api(client):
    a = APIClient("http://testserver", client.headers["Authorization"].split()[1])
    a._http = client  # the FastAPI TestClient is an httpx.Client: same request path, no socket
    return a


@pytest.fixture
def dc(api):
    return Client(api, "main")


def test_backends_collection(dc):
    assert [b.name for b in dc.backends.list()] == [] or all(b.name for b in dc.backends.list())
    b = dc.backends.create({"type": "vultr", "creds": {"type": "api_key", "api_key": "secret-key"}})
    assert b.name == "vultr" and "creds" not in b.config
    assert "secret-key" not in repr(dc.backends.list()) + str([x.config for x in dc.backends.list()])
    with pytest.raises(ServerClientError):
        dc.backends.create({"type": "vultr", "creds": {"type": "api_key", "api_key": "k2"}})  # exists
    dc.backends.delete(["vultr"])
    assert "vultr" not in [x.name for x in dc.backends.list()]


def test_fleet_and_volume_collections(dc):
    from dstack_amd.core.models.fleets import FleetConfiguration
    from dstack_amd.core.models.volumes import VolumeConfiguration

    key = {"public": "ssh-ed25519 AAAA", "private": "-----BEGIN OPENSSH PRIVATE KEY-----\nx\n"
                                                   "-----END OPENSSH PRIVATE KEY-----\n"}
    conf = FleetConfiguration.model_validate({"type": "fleet", "name": "onprem", "ssh_config": {
        "user": "ubuntu", "ssh_key": key, "hosts": ["10.0.0.1", "10.0.0.2"]}})
    fleet = dc.fleets.apply_configuration(conf)
    assert fleet.name == "onprem" and len(fleet.instances) == 2
    assert [f.name for f in dc.fleets.list()] == ["onprem"]
    assert dc.fleets.get("onprem").id == fleet.id
    dc.fleets.delete("onprem")

    vol = dc.volumes.create(VolumeConfiguration.model_validate(
        {"type": "volume", "name": "data", "backend": "local", "region": "local", "size": "100GB"}))
    assert vol.name == "data" and [v.name for v in dc.volumes.list()] == ["data"]
    assert dc.volumes.get("data").id == vol.id
    dc.volumes.delete("data")


def test_runs_plan_submit_list_stop(dc):
    task = Task(commands=["echo hi"], resources=Resources(gpu=GPU(name=["MI355X"], count=8)))
    plan = dc.runs.get_plan(task, VirtualRepo(), run_name="api-run")
    assert plan.run_spec.run_name == "api-run"
    assert plan.run_spec.configuration.resources.gpu.vendor.value == "amd"
    run = dc.runs.exec_plan(plan, VirtualRepo())
    assert run.name == "api-run" and run.status.value == "submitted"
    assert [r.name for r in dc.runs.list()] == ["api-run"]
    got = dc.runs.get("api-run")
    assert got is not None and got.model.id == run.model.id
    assert dc.runs.get("nope") is None
    got.stop()
    assert dc.runs.get("api-run").status.value in ("terminating", "terminated", "done", "aborted")


def test_users_and_projects_via_api_client(api):
    me = api.users.get_my_user()
    assert me.username == "admin" and me.global_role.value == "admin"
    u = api.users.create("alice", global_role="user")
    assert u.username == "alice"
    p = api.projects.create("team")
    assert p.project_name == "team"
    p = api.projects.set_members("team", [{"username": "alice", "project_role": "manager"},
                                          {"username": "admin", "project_role": "admin"}])
    assert {m.user.username: m.project_role.value for m in p.members} == {"alice": "manager", "admin": "admin"}
    api.projects.delete(["team"])
    assert "team" not in [x.project_name for x in api.projects.list()]
    api.users.delete(["alice"])
    assert "alice" not in [x.username for x in api.users.list()]


def test_service_url_and_model_and_offers(dc):
    from dstack_amd.api import OpenAIChatModel, Service
    from dstack_amd.core.models.profiles import Profile
    from dstack_amd.core.models.resources import ResourcesSpec
    from dstack_amd.core.models.runs import Requirements

    svc = Service(commands=["python3 -m http.server 8000"], port=8000, name="api-svc",
                  model=OpenAIChatModel(name="llama", format="openai"))
    run = dc.runs.submit(svc, VirtualRepo())
    assert run.service_url == "http://testserver/proxy/services/main/api-svc/"
    m = run.service_model
    assert m.name == "llama" and m.url == "http://testserver/proxy/models/main/"
    task = dc.runs.submit(Task(commands=["true"], name="api-task"), VirtualRepo())
    with pytest.raises(ValueError):
        task.service_model
    offers = dc.runs.get_offers(Profile(name="p"), Requirements(resources=ResourcesSpec()))
    assert offers.instances and all(o.backend.value == "local" for o in offers.instances)


def test_repo_collection_load(dc, tmp_path, monkeypatch):
    from dstack_amd.core.errors import ConfigurationError
    from dstack_amd.core.models.repos import LocalRepo

    monkeypatch.setenv("DSTACK_DIR", str(tmp_path / "home"))
    work = tmp_path / "work"
    work.mkdir()
    (work / "train.py").write_text("print(1)\n")
    with pytest.raises(ConfigurationError):
        dc.repos.load(str(work))
    repo = dc.repos.load(str(work), init=True)
    assert isinstance(repo, LocalRepo) and dc.repos.is_initialized(repo)
    again = dc.repos.load(str(work))
    assert isinstance(again, LocalRepo) and again.repo_id == repo.repo_id


def test_pool_collection_legacy_api(dc):
    """(reference ``api/_public/pools.py``) the deprecated ``client.pool`` still lists, creates,
    shows and deletes pools."""
    names = [p.name for p in dc.pool.list()]
    assert names  # the project's default pool is created on first listing
    p = dc.pool.create("legacy")
    assert p.name == "legacy" and repr(p) == "<PoolInstance 'legacy'>" and p.total_instances == 0
    assert dc.pool.show("legacy").name == "legacy"
    dc.pool.delete("legacy")
    assert "legacy" not in [x.name for x in dc.pool.list()]


def test_sft_fine_tuning_task_builds_a_runnable_task(dc, tmp_path):
    """``SFTFineTuningTask`` (reference ``api/huggingface``) is a Task whose commands install the HF
    stack, unpack the shipped training script and launch it once per GPU with the given options."""
    import base64
    import py_compile

    from dstack_amd.api.huggingface import SFTFineTuningTask

    with pytest.raises(ValueError, match="HF_TOKEN"):
        SFTFineTuningTask(model_name="m", dataset_name="d", env={})
    t = SFTFineTuningTask(model_name="meta-llama/Llama-3.1-8B", dataset_name="org/sft data", env={"HF_TOKEN": "x"},
                          lora_r=16, max_steps=10, use_4bit=True, resources={"gpu": "MI355X:8"})
    assert t.type == "task" and t.sft_args["lora_r"] == 16
    install, unpack, launch = t.commands
    assert "trl" in install and "bitsandbytes" in install
    blob = unpack.split()[1]
    script = tmp_path / "sft.py"
    script.write_bytes(base64.b64decode(blob))
    py_compile.compile(str(script), doraise=True)
    assert launch.startswith("accelerate launch --num_processes ${DSTACK_GPUS_PER_NODE:-1}")
    assert "--lora_r 16" in launch and "--max_steps 10" in launch and "'org/sft data'" in launch
    # the script's CLI accepts exactly what the task passes
    import importlib.util
    import shlex

    spec = importlib.util.spec_from_file_location("sft_script", script)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    parsed = mod.parse_args(shlex.split(launch.split("/tmp/dstack_sft_train.py", 1)[1]))
    assert parsed.lora_r == 16 and parsed.use_4bit is True and parsed.dataset_name == "org/sft data"
    # and the server accepts it as a run configuration
    plan = dc.runs.get_plan(t)
    assert plan.job_plans and plan.job_plans[0].job_spec.commands[-1].endswith(launch)
