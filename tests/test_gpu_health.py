"""GPU health probing off the job path.

* The native shim runs ``dstack-probe --quick --json`` asynchronously after it starts (and on
  ``POST /api/gpu_health/probe``), holding the GPUs in its lock meanwhile, and serves the result on
  ``GET /api/gpu_health``; tested with the real shim binary, a fake /sys tree (two MI355X render
  nodes) and a stand-in probe script.
* The server copies that result into the instance's health (relative per-SKU thresholds decided by
  the probe) at registration and while the host idles, re-probes stale results only on idle hosts,
  and the scheduler skips hosts whose GPUs failed.
"""

from __future__ import annotations

import json
import os
import subprocess
import time
from unittest import mock

import httpx
import pytest

from dstack_amd import native_bin
from dstack_amd.core.models.instances import InstanceStatus
from dstack_amd.server.background.tasks import process_instances as pi
from dstack_amd.server.db import session_scope
from dstack_amd.server.models import InstanceModel

from tests.test_reconcilers import _instance, _jpd

GOOD = {"sku": "MI355X", "baseline": {"hbm_tb_s": 6.0, "mfma_bf16_tflops": 2100},
        "thresholds": {"hbm_tb_s": 4.8, "mfma_bf16_tflops": 1680}, "hbm_tb_s": [6.05, 6.01],
        "mfma_bf16_tflops": [2098.0, 2101.5], "mfma_fp8_tflops": [4970.0, 4981.0], "devices": 2,
        "healthy": True, "message": ""}
BAD = dict(GOOD, hbm_tb_s=[6.05, 3.10], healthy=False, message="GPU 1 HBM TB/s 3.10 < 4.80")


def _fake_sysfs(root):
    for render, bdf in ((128, "0000:75:00.0"), (136, "0000:05:00.0")):
        dev = root / "devices" / bdf
        dev.mkdir(parents=True)
        (dev / "vendor").write_text("0x1002\n")
        (dev / "product_name").write_text("AMD Instinct MI355X\n")
        (dev / "mem_info_vram_total").write_text(str(288 << 30) + "\n")
        d = root / "sys" / "class" / "drm" / f"renderD{render}"
        d.mkdir(parents=True)
        os.symlink(dev, d / "device")
        (root / "dev" / "dri").mkdir(parents=True, exist_ok=True)
        (root / "dev" / "dri" / f"renderD{render}").write_text("")


@pytest.fixture
def shim(tmp_path):
    shim_bin = native_bin.shim_path()
    if not shim_bin:
        pytest.skip("native agents not built")
    _fake_sysfs(tmp_path / "fs")
    probe = tmp_path / "fake-probe"
    # a stand-in for dstack-probe: takes a moment (the GPUs are held meanwhile), prints the document
    probe.write_text("#!/bin/sh\nsleep 0.6\necho 'running probes...'\n"
                     f"echo '{json.dumps(GOOD)}'\n")
    probe.chmod(0o755)
    env = dict(os.environ, DSTACK_SYSFS_ROOT=str(tmp_path / "fs"), HOME=str(tmp_path))
    p = subprocess.Popen([shim_bin, "--shim-home", str(tmp_path / "home"), "--shim-http-port", "0", "--host",
                          "127.0.0.1", "--driver", "process", "--probe-binary", str(probe),
                          "--runner-binary-path", "/bin/true"], stdout=subprocess.PIPE, stderr=subprocess.DEVNULL,
                         text=True, env=env, start_new_session=True)
    try:
        line = p.stdout.readline()
        assert line.startswith("DSTACK_SHIM_PORT="), line
        yield f"http://127.0.0.1:{int(line.split('=')[1])}", probe
    finally:
        p.terminate()
        p.wait(10)


def _wait_state(url, states, timeout=10):
    deadline = time.time() + timeout
    while time.time() < deadline:
        d = httpx.get(url + "/api/gpu_health", timeout=2).json()
        if d["state"] in states:
            return d
        time.sleep(0.05)
    raise AssertionError(f"gpu_health never reached {states}: {d}")


def test_shim_probes_at_start_and_on_demand(shim):
    url, probe = shim
    hc = httpx.get(url + "/api/healthcheck", timeout=2).json()
    assert hc["gpus_total"] == 2 and hc["gpu_health"] in ("running", "done")
    d = _wait_state(url, {"done"})
    assert d["result"]["healthy"] is True and d["result"]["sku"] == "MI355X"
    assert d["ran_at_ms"] >= d["started_at_ms"] > 0
    # on demand: a new run with a new timestamp; the GPUs are held while it runs
    probe.write_text(probe.read_text().replace(json.dumps(GOOD), json.dumps(BAD)))
    r = httpx.post(url + "/api/gpu_health/probe", timeout=2)
    assert r.status_code == 202 and r.json()["state"] == "started"
    assert httpx.get(url + "/api/healthcheck", timeout=2).json()["gpus_free"] == 0
    d2 = _wait_state(url, {"done"})
    assert d2["ran_at_ms"] > d["ran_at_ms"] and d2["result"]["healthy"] is False
    assert httpx.get(url + "/api/healthcheck", timeout=2).json()["gpus_free"] == 2


def test_gpu_task_preempts_a_running_probe(shim, tmp_path):
    """A task asking for GPUs while the probe holds them pre-empts it: the probe is killed (state
    "interrupted"), the task gets its GPU at once instead of waiting out the probe, and the probe
    runs again once the host is idle."""
    url, probe = shim
    _wait_state(url, {"done"})
    first = httpx.get(url + "/api/gpu_health", timeout=2).json()
    marker = tmp_path / "probe-finished"
    runs = tmp_path / "probe-runs"
    probe.write_text("#!/bin/sh\n"
                     f"echo run >> {runs}\n"
                     "sleep 30\n"
                     f"touch {marker}\n"
                     f"echo '{json.dumps(GOOD)}'\n")
    assert httpx.post(url + "/api/gpu_health/probe", timeout=2).json()["state"] == "started"
    deadline = time.time() + 5
    while not runs.exists() and time.time() < deadline:
        time.sleep(0.02)
    assert httpx.get(url + "/api/healthcheck", timeout=2).json()["gpus_free"] == 0
    t0 = time.time()
    r = httpx.post(url + "/api/tasks", json={"id": "t1", "name": "t1", "image_name": "x", "gpu": 1,
                                            "container_ssh_keys": []}, timeout=5)
    assert r.status_code == 200
    t = {}
    while time.time() < t0 + 10:
        t = httpx.get(url + "/api/tasks/t1", timeout=2).json()
        if t.get("gpus"):
            break
        time.sleep(0.01)
    granted_after = time.time() - t0
    assert t.get("gpus") and len(t["gpus"]) == 1, t
    assert granted_after < 1.0, granted_after  # not behind the 30 s probe
    h = httpx.get(url + "/api/gpu_health", timeout=2).json()
    assert h["state"] in ("interrupted", "running"), h  # running = already re-probing after the task
    assert h["ran_at_ms"] == first["ran_at_ms"] or h["state"] == "running"
    assert not marker.exists()  # killed, never finished
    assert t["render_nodes"] == [["/dev/dri/renderD136", "/dev/dri/renderD128"][t["gpus"][0]]]
    # the task ends (stand-in runner): the host is idle again and the interrupted probe re-runs
    deadline = time.time() + 20
    while time.time() < deadline and runs.read_text().count("run") < 2:
        time.sleep(0.05)
    assert runs.read_text().count("run") == 2


def test_probe_and_task_never_share_gpus(shim):
    """Interleaved probe requests and GPU tasks: a probe that finds a GPU in use reports "busy"
    and never starts beside the job; a task never fails because the probe held the GPUs."""
    url, _ = shim
    _wait_state(url, {"done"})
    states, tasks = [], []
    for i in range(6):
        states.append(httpx.post(url + "/api/gpu_health/probe", timeout=2).json()["state"])
        tid = f"mix{i}"
        httpx.post(url + "/api/tasks", json={"id": tid, "name": tid, "image_name": "x", "gpu": 1,
                                            "container_ssh_keys": []}, timeout=5)
        tasks.append(tid)
    deadline = time.time() + 20
    final = {}
    while time.time() < deadline:
        final = {tid: httpx.get(url + f"/api/tasks/{tid}", timeout=2).json() for tid in tasks}
        if all(t["status"] == "terminated" for t in final.values()):
            break
        time.sleep(0.05)
    for t in final.values():
        assert t.get("termination_message") != "not enough free GPUs", t
        assert t.get("termination_message") != "requested GPUs are busy", t
    assert set(states) <= {"started", "running", "busy"}


# ---- server side -----------------------------------------------------------------------------
class FakeShim:
    def __init__(self, doc):
        self.doc = doc
        self.started = 0

    def gpu_health(self):
        return self.doc

    def start_gpu_probe(self):
        self.started += 1
        return "started"

    def healthcheck(self):
        return {"service": "dstack-shim"}


def _doc(result, ran_at):
    return {"state": "done", "started_at_ms": int(ran_at * 1000) - 500, "ran_at_ms": int(ran_at * 1000),
            "result": result}


def test_registration_records_probe_and_scheduler_skips_bad_host(db):
    from dstack_amd.core.models.profiles import Profile
    from dstack_amd.core.models.runs import Requirements
    from dstack_amd.core.models.resources import ResourcesSpec
    from dstack_amd.server.services import pools as pools_services

    now = time.time()
    with session_scope() as s:
        iid = _instance(s, status=InstanceStatus.PROVISIONING)
    fake = FakeShim(_doc(BAD, now))
    with mock.patch.object(pi, "get_shim_client", return_value=fake), session_scope() as s:
        inst = s.get(InstanceModel, iid)
        pi._check_provisioning(s, inst)
        assert inst.status == InstanceStatus.IDLE.value
        h = json.loads(inst.health_data)
        assert h["healthy"] is False and h["source"] == "shim" and h["sku"] == "MI355X"
        assert h["thresholds"]["hbm_tb_s"] == 4.8 and "GPU 1 HBM" in inst.health_status
        req = Requirements(resources=ResourcesSpec.model_validate({"gpu": "MI355X:1"}))
        assert pools_services.filter_pool_instances([inst], Profile(name="p"), req) == []
    assert fake.started == 0  # a fresh result: no re-probe
    # the host is repaired and re-probed: healthy again, schedulable again
    fake.doc = _doc(GOOD, now + 10)
    with mock.patch.object(pi, "get_shim_client", return_value=fake), session_scope() as s:
        inst = s.get(InstanceModel, iid)
        pi._health_polled.clear()
        pi._check_instance(s, inst)
        assert json.loads(inst.health_data)["healthy"] is True
    with session_scope() as s:
        assert s.get(InstanceModel, iid).health_status in (None, "")


def test_stale_result_reprobed_only_on_idle_hosts(db):
    old = time.time() - 7 * 3600
    with session_scope() as s:
        idle = _instance(s, status=InstanceStatus.IDLE)
        busy = _instance(s, status=InstanceStatus.BUSY)
        s.get(InstanceModel, busy).busy_blocks = 1
    fake = FakeShim(_doc(GOOD, old))
    with mock.patch.object(pi, "get_shim_client", return_value=fake), session_scope() as s:
        pi._health_polled.clear()
        pi.refresh_gpu_health(s.get(InstanceModel, busy), _jpd())
        assert fake.started == 0  # a job runs there: the probe would disturb it
        pi.refresh_gpu_health(s.get(InstanceModel, idle), _jpd())
        assert fake.started == 1
        # polled at most once a minute
        pi.refresh_gpu_health(s.get(InstanceModel, idle), _jpd())
        assert fake.started == 1


# ---- on the MI355X --------------------------------------------------------------------------------
@pytest.mark.gpu
def test_real_probe_relative_thresholds_and_one_rank_rccl():
    """dstack-probe on the real GPU: MI355X baseline detected, thresholds = 80 % of it, healthy; the
    RCCL path (ncclCommInitRank from a unique id, the job's bootstrap) runs with one rank."""
    probe = native_bin.probe_path()
    assert probe, "dstack-probe must be built for GPU runs"
    r = subprocess.run([probe, "--quick", "--json", "--hbm", "--mfma"], capture_output=True, text=True, timeout=180)
    doc = json.loads(r.stdout.strip().splitlines()[-1])
    print(doc)
    assert doc["sku"] == "MI355X"
    assert doc["thresholds"]["hbm_tb_s"] == pytest.approx(0.8 * doc["baseline"]["hbm_tb_s"], rel=1e-3)
    assert doc["healthy"] is True and r.returncode == 0, doc
    assert min(doc["hbm_tb_s"]) >= doc["thresholds"]["hbm_tb_s"]
    assert min(doc["mfma_bf16_tflops"]) >= doc["thresholds"]["mfma_bf16_tflops"]
    # one process per GPU, forked before the probe touches HIP; at world 1 the sweep proves the
    # bootstrap + communicator + an exact fp32 sum, and is flagged as not a bandwidth measurement
    r = subprocess.run([probe, "--rccl", "--quick", "--json"], capture_output=True, text=True, timeout=180)
    doc = json.loads(r.stdout.strip().splitlines()[-1])
    print(doc)
    assert r.returncode == 0 and doc["healthy"] is True, doc
    assert doc["rccl_world"] == doc["rccl_gpus_per_node"] >= 1 and len(doc["rccl"]) >= 4
    assert all(x["algbw_gb_s"] > 0 for x in doc["rccl"])
    if doc["rccl_world"] == 1:
        assert doc["rccl_busbw_gb_s"] is None and "not a bandwidth measurement" in doc["rccl_note"]
    else:
        assert doc["rccl_busbw_gb_s"] > 0


@pytest.mark.gpu
def test_shim_startup_probe_on_gpu(tmp_path):
    """The shim probes the real GPU right after it starts, off any job path, and serves the result."""
    shim_bin, probe = native_bin.shim_path(), native_bin.probe_path()
    assert shim_bin and probe
    p = subprocess.Popen([shim_bin, "--shim-home", str(tmp_path / "home"), "--shim-http-port", "0", "--host",
                          "127.0.0.1", "--driver", "process", "--probe-binary", probe, "--runner-binary-path",
                          "/bin/true"], stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True,
                         start_new_session=True)
    try:
        line = p.stdout.readline()
        url = f"http://127.0.0.1:{int(line.split('=')[1])}"
        d = _wait_state(url, {"done", "failed"}, timeout=150)
        print(d)
        assert d["state"] == "done" and d["result"]["healthy"] is True and d["result"]["sku"] == "MI355X"
        assert httpx.get(url + "/api/healthcheck", timeout=2).json()["gpus_free"] >= 1
    finally:
        p.terminate()
        p.wait(10)


@pytest.mark.gpu
def test_gpu_discovery_paths_agree_with_hip_order():
    """amdsmi and sysfs discovery list the same GPUs in the same (PCI BDF) order, and that order is
    the HIP device order torch sees -- so a GPU-lock index, its xGMI row and its render node agree."""
    import torch

    out = subprocess.run([native_bin.shim_path(), "--list-gpus"], capture_output=True, text=True, timeout=60)
    d = json.loads(out.stdout.strip().splitlines()[-1])
    print(d)
    smi, sysfs = d["amdsmi"], d["sysfs"]
    assert smi, "amdsmi sees no GPU"
    assert [g["bdf"] for g in smi] == [g["bdf"] for g in sysfs]
    assert [g["render_node"] for g in smi] == [g["render_node"] for g in sysfs]
    assert [g["bdf"] for g in smi] == sorted(g["bdf"] for g in smi)
    n = torch.cuda.device_count()
    assert n == len(smi)
    for i in range(n):
        pr = torch.cuda.get_device_properties(i)
        if hasattr(pr, "pci_bus_id"):
            assert int(smi[i]["bdf"].split(":")[1], 16) == pr.pci_bus_id, (i, smi[i]["bdf"], pr.pci_bus_id)


def test_failed_driver_bootstrap_fails_provisioning_with_its_reason(db):
    """A GPU offer whose host came up without /dev/kfd (the cloud bootstrap's amdgpu install failed,
    core/backends/base.py marker -> shim host_info ``gpu_driver_error``) is not registered as an
    idle host with zero GPUs: provisioning fails with the bootstrap's reason."""
    msg = "amdgpu 7.0 driver install failed on ubuntu/noble kernel 6.8.0-45-generic: /dev/kfd missing"

    class NoDriverShim(FakeShim):
        def host_info(self):
            return {"gpu_count": 0, "gpu_vendor": "", "gpu_driver_error": msg}

    with session_scope() as s:
        iid = _instance(s, status=InstanceStatus.PROVISIONING)
    with mock.patch.object(pi, "get_shim_client", return_value=NoDriverShim(None)), session_scope() as s:
        inst = s.get(InstanceModel, iid)
        pi._check_provisioning(s, inst)
        assert inst.status == InstanceStatus.TERMINATING.value
        assert inst.termination_reason == f"GPU driver: {msg}" and inst.health_status == inst.termination_reason

    class DriverOkShim(FakeShim):
        def host_info(self):  # a marker left from an earlier boot does not matter once GPUs are up
            return {"gpu_count": 8, "gpu_vendor": "amd", "gpu_driver_error": msg}

    with session_scope() as s:
        iid = _instance(s, status=InstanceStatus.PROVISIONING)
    with mock.patch.object(pi, "get_shim_client", return_value=DriverOkShim(_doc(GOOD, time.time()))), \
            session_scope() as s:
        inst = s.get(InstanceModel, iid)
        pi._check_provisioning(s, inst)
        assert inst.status == InstanceStatus.IDLE.value
