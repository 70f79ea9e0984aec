"""Server services without their own router tests: encryption keys and rotation, the server config
manager, job metrics from stored points and their collection task, and the CLI's port lock and SSH
config editor.

Reference behaviour: ``S/services/encryption/__init__.py:38-102``, ``S/services/config.py:519-676``,
``S/services/metrics.py:54-104``, ``C/services/ssh/ports.py:17-84``, ``C/services/ssh/attach.py``.
"""

import json
import socket

import pytest
import yaml
from sqlalchemy import text

from dstack_amd.server.db import session_scope
from dstack_amd.server.models import BackendModel, JobModel, JobMetricsPoint, ProjectModel, UserModel
from dstack_amd.server.services import encryption


@pytest.fixture
def keys():
    yield
    encryption.configure_keys(None)


def _aes(name):
    return {"type": "aes", "name": name, "secret": encryption.generate_aes_key()}


def test_aes_roundtrip_and_payload_is_not_plaintext(keys):
    encryption.configure_keys([_aes("k1")])
    enc = encryption.encrypt("s3cret-token")
    assert enc.startswith("enc:aes:k1:") and "s3cret" not in enc
    assert encryption.decrypt(enc) == "s3cret-token"
    # fresh nonce per value
    assert encryption.encrypt("s3cret-token") != enc


def test_key_rotation_reads_old_values_and_writes_with_first_key(keys):
    old = _aes("old")
    encryption.configure_keys([old])
    enc_old = encryption.encrypt("v")
    encryption.configure_keys([_aes("new"), old])
    assert encryption.decrypt(enc_old) == "v"
    assert encryption.encrypt("v").startswith("enc:aes:new:")
    encryption.configure_keys([_aes("new")])
    with pytest.raises(encryption.EncryptionError):
        encryption.decrypt(enc_old)


def test_identity_and_legacy_plaintext(keys):
    encryption.configure_keys(None)
    enc = encryption.encrypt("x")
    assert enc.startswith("enc:identity:")
    assert encryption.decrypt(enc) == "x"
    assert encryption.decrypt("plain-legacy") == "plain-legacy"
    # identity-encoded values stay readable after an AES key is added
    encryption.configure_keys([_aes("k")])
    assert encryption.decrypt(enc) == "x"


def test_bad_aes_key_length_rejected(keys):
    with pytest.raises(encryption.EncryptionError):
        encryption.configure_keys([{"type": "aes", "name": "k", "secret": "c2hvcnQ="}])


def test_server_config_creates_projects_backends_and_encrypts_creds(db, tmp_path, keys):
    from dstack_amd.server.services.config import ServerConfigManager

    cfg = {
        "projects": [{"name": "team", "backends": [
            {"type": "vultr", "creds": {"type": "api_key", "api_key": "VULTR-KEY"}}]}],
        "encryption": {"keys": [_aes("main")]},
    }
    path = tmp_path / "config.yml"
    path.write_text(yaml.safe_dump(cfg))
    m = ServerConfigManager(path)
    assert m.load_config()
    m.apply_encryption()
    with session_scope() as s:
        admin = s.query(UserModel).filter_by(name="admin").one()
        m.apply_config(s, admin)
    # applying again updates instead of failing on the existing backend
    cfg["projects"][0]["backends"][0]["regions"] = ["ewr"]
    path.write_text(yaml.safe_dump(cfg))
    m.load_config()
    with session_scope() as s:
        m.apply_config(s, s.query(UserModel).filter_by(name="admin").one())
    with session_scope() as s:
        project = s.query(ProjectModel).filter_by(name="team").one()
        (b,) = s.query(BackendModel).filter_by(project_id=project.id).all()
        assert json.loads(b.auth)["api_key"] == "VULTR-KEY"
        assert json.loads(b.config)["regions"] == ["ewr"]
        raw = s.execute(text("SELECT auth FROM backends WHERE id = :i"), {"i": str(b.id)}).scalar_one()
        assert raw.startswith("enc:aes:main:") and "VULTR-KEY" not in raw


def test_server_config_missing_file_is_noop(tmp_path):
    from dstack_amd.server.services.config import ServerConfigManager

    m = ServerConfigManager(tmp_path / "absent.yml")
    assert not m.load_config()
    m.init_config("main")
    assert yaml.safe_load((tmp_path / "absent.yml").read_text())["projects"][0]["name"] == "main"


def _job(s):
    from dstack_amd.core.models.runs import RunSpec
    from dstack_amd.server.services import runs as runs_services

    project = s.query(ProjectModel).filter_by(name="main").one()
    user = s.query(UserModel).filter_by(name="admin").one()
    spec = RunSpec.model_validate({"run_name": "m1", "repo_id": "virt", "repo_data": {"repo_type": "virtual"},
                                   "configuration": {"type": "task", "commands": ["x"]}, "ssh_key_pub": ""})
    run = runs_services.submit_run(s, project, user, spec)
    return s.query(JobModel).filter_by(run_id=run.id).one()


def _point(ts_s, cpu_us, util):
    return {"timestamp_micro": int(ts_s * 1e6), "cpu_usage_micro": cpu_us, "memory_usage_bytes": 10 << 30,
            "memory_working_set_bytes": 8 << 30,
            "gpus": [{"gpu_memory_usage_bytes": 100 << 30, "gpu_util_percent": u, "gpu_power_watts": 1000,
                      "gpu_temperature_c": 60} for u in util]}


def test_job_metrics_from_last_points(db):
    from dstack_amd.server.services import metrics

    with session_scope() as s:
        job = _job(s)
        assert metrics.get_job_metrics(s, job).metrics == []
        metrics.store_metrics_point(s, job, _point(100, 0, [0, 0]))
        # 10 s later: 25 CPU-seconds used -> 250 %
        metrics.store_metrics_point(s, job, _point(110, 25_000_000, [97, 99]))
        s.flush()
        by_name = {m.name: m.values for m in metrics.get_job_metrics(s, job).metrics}
    assert by_name["cpu_usage_percent"] == [pytest.approx(250.0)]
    assert by_name["gpus_detected_num"] == [2.0]
    assert by_name["gpu_util_percent_gpu0"] == [97.0] and by_name["gpu_util_percent_gpu1"] == [99.0]
    assert by_name["memory_working_set_bytes"] == [float(8 << 30)]
    assert by_name["gpu_power_watts_gpu1"] == [1000.0]


def test_xgmi_and_hbm_metrics(db):
    """amdsmi xGMI counters are cumulative KiB per GPU: the server reports the rate between two
    samples, links up, and the HBM controller activity; Prometheus exposes the raw counters."""
    from dstack_amd.server.services import metrics, prometheus

    def pt(ts, read_kb, write_kb, up):
        p = _point(ts, 0, [50])
        p["gpus"][0]["gpu_mem_activity_percent"] = 71
        p["gpus"][0]["xgmi"] = {"links_total": 7, "links_up": up, "link_speed_gbps": 32, "link_width": 16,
                                "read_kb": read_kb, "write_kb": write_kb}
        return p

    with session_scope() as s:
        job = _job(s)
        metrics.store_metrics_point(s, job, pt(100, 1_000, 0, 7))
        metrics.store_metrics_point(s, job, pt(102, 1_000 + 2 * 1024 * 1024, 512, 6))
        s.flush()
        by_name = {m.name: m.values for m in metrics.get_job_metrics(s, job).metrics}
        job.status = "running"
        s.flush()
        text = prometheus.render(s)
    assert by_name["gpu_xgmi_read_bytes_per_s_gpu0"] == [pytest.approx(1024 ** 3)]  # 2 GiB in 2 s
    assert by_name["gpu_xgmi_write_bytes_per_s_gpu0"] == [pytest.approx(512 * 1024 / 2)]
    assert by_name["gpu_xgmi_links_up_gpu0"] == [6.0]
    assert by_name["gpu_hbm_activity_percent_gpu0"] == [71.0]
    assert 'dstack_job_gpu_xgmi_links_up{run="m1"' in text
    assert f"dstack_job_gpu_xgmi_read_bytes_total" in text and str((1_000 + 2 * 1024 * 1024) * 1024) in text


def test_metrics_ttl_cleanup(db):
    from dstack_amd.server.services import metrics

    with session_scope() as s:
        job = _job(s)
        metrics.store_metrics_point(s, job, _point(1000, 0, [0]))
        metrics.store_metrics_point(s, job, _point(5000, 0, [0]))
        s.flush()
        metrics.delete_old_metrics(s, ttl_seconds=3600, now_micro=int(5000 * 1e6))
        left = [p.timestamp_micro for p in s.query(JobMetricsPoint).filter_by(job_id=job.id)]
    assert left == [int(5000 * 1e6)]


def _free_port():
    with socket.socket() as t:
        t.bind(("127.0.0.1", 0))
        return t.getsockname()[1]


def test_ports_lock_honours_requests_and_detects_conflicts():
    from dstack_amd.core.services.ssh.ports import PortsLock, PortUsedError

    want = _free_port()
    lock = PortsLock({8000: want, 9000: 0}).acquire()
    mapping = lock.dict()
    assert mapping[8000] == want and mapping[9000] not in (0, want)
    # a held port cannot be taken by a second lock
    with pytest.raises(PortUsedError):
        PortsLock({1: want}).acquire()
    assert lock.release() == mapping
    PortsLock({1: want}).acquire().release()
    with pytest.raises(PortUsedError):
        PortsLock({1: want, 2: want}).acquire()


def test_ssh_config_blocks_added_replaced_removed(tmp_path, monkeypatch):
    from dstack_amd.core.services.ssh import attach

    cfg = tmp_path / "ssh" / "config"
    monkeypatch.setattr(attach, "ssh_config_path", lambda: cfg)
    attach.update_ssh_config("run-host", {"HostName": "1.2.3.4", "Port": 22})
    attach.update_ssh_config("run", {"HostName": "localhost", "ProxyJump": "run-host"})
    attach.update_ssh_config("run-host", {"HostName": "5.6.7.8", "Port": 22})
    text_ = cfg.read_text()
    assert text_.count("Host run-host") == 1 and "5.6.7.8" in text_ and "1.2.3.4" not in text_
    assert "ProxyJump run-host" in text_
    attach.update_ssh_config("run", None)
    assert "Host run\n" not in cfg.read_text() and "Host run-host" in cfg.read_text()
    attach.update_ssh_config("run-host", None)
    assert cfg.read_text() == ""


def test_collect_metrics_polls_running_jobs_only(db):
    from unittest import mock

    from dstack_amd.server.background.tasks import process_metrics
    from dstack_amd.server.services import metrics

    from tests.test_reconcilers import _jpd

    with session_scope() as s:
        job = _job(s)
        job_id = job.id
        job.status = "running"
        job.job_provisioning_data = _jpd().model_dump_json()
    client = mock.Mock()
    client.get_metrics.side_effect = [_point(100, 0, [50]), _point(101, 1_000_000, [60])]
    with mock.patch.object(process_metrics, "get_runner_client", return_value=client) as factory:
        process_metrics.collect_metrics()
        process_metrics.collect_metrics()
    assert factory.call_count == 2
    with session_scope() as s:
        job = s.get(JobModel, job_id)
        by_name = {m.name: m.values for m in metrics.get_job_metrics(s, job).metrics}
        assert by_name["cpu_usage_percent"] == [pytest.approx(100.0)]
        assert by_name["gpu_util_percent_gpu0"] == [60.0]
        job.status = "done"
    client.get_metrics.side_effect = AssertionError("finished jobs are not polled")
    with mock.patch.object(process_metrics, "get_runner_client", return_value=client):
        process_metrics.collect_metrics()


def test_attach_retries_until_the_container_sshd_is_up(tmp_path, monkeypatch):
    """The container bootstrap execs the runner first and starts sshd in the background, so the
    first attach may find the port closed: ssh is retried (exit 255) until it connects (the
    ControlPersist master exits 0), and gives up with the ssh error after DSTACK_ATTACH_TIMEOUT."""
    import types

    from dstack_amd.core.errors import SSHError
    from dstack_amd.core.services.ssh import attach

    monkeypatch.setattr(attach, "ssh_config_path", lambda: tmp_path / "ssh" / "config")
    bin_dir = tmp_path / "bin"
    bin_dir.mkdir()
    count = tmp_path / "count"
    (bin_dir / "ssh").write_text(
        "#!/bin/sh\n"
        f"n=$(cat {count} 2>/dev/null || echo 0); n=$((n + 1)); echo $n > {count}\n"
        "case \"$*\" in *'-O exit'*) exit 0;; esac\n"
        "if [ $n -le 2 ]; then echo 'ssh: connect to host 10.0.0.5 port 10022: Connection refused' >&2; exit 255; fi\n"
        "exit 0\n")
    (bin_dir / "ssh").chmod(0o755)
    monkeypatch.setenv("PATH", f"{bin_dir}:/usr/bin:/bin")
    conf = types.SimpleNamespace(ports=[], type="task")
    run = types.SimpleNamespace(run_spec=types.SimpleNamespace(run_name="r1", configuration=conf))
    jpd = types.SimpleNamespace(backend=types.SimpleNamespace(value="aws"), hostname="10.0.0.5", ssh_port=10022,
                                username="root")
    sub = types.SimpleNamespace(job_provisioning_data=jpd, job_runtime_data=None)
    a = attach.RunAttach(run, sub, identity_file=str(tmp_path / "id"))
    a.open()
    assert count.read_text().strip() == "3"  # two refusals, then connected
    a.close()
    count.write_text("-100")  # every attempt refused
    monkeypatch.setenv("DSTACK_ATTACH_TIMEOUT", "1")
    b = attach.RunAttach(run, sub, identity_file=str(tmp_path / "id"))
    with pytest.raises(SSHError, match="Connection refused"):
        b.open()


def _apply(m, path, cfg):
    path.write_text(yaml.safe_dump(cfg))
    m.load_config()
    with session_scope() as s:
        m.apply_config(s, s.query(UserModel).filter_by(name="admin").one())


def _backend_types(name):
    with session_scope() as s:
        project = s.query(ProjectModel).filter_by(name=name).one()
        return sorted(b.type for b in s.query(BackendModel).filter_by(project_id=project.id).all())


def test_server_config_deletes_unlisted_skips_unchanged_and_survives_a_bad_backend(db, tmp_path, keys, monkeypatch):
    """Reference ``services/config.py:560-616``: a backend dropped from config.yml is deleted, an
    unchanged one is not re-validated or rewritten, and one invalid backend is logged and skipped
    while the valid ones next to it are configured."""
    from dstack_amd.server.services import backends as backends_services
    from dstack_amd.server.services.config import ServerConfigManager

    checks = []
    real = backends_services.validate_credentials
    monkeypatch.setattr(backends_services, "validate_credentials",
                        lambda btype, cfg, secrets: (checks.append(btype.value), real(btype, cfg, secrets)))
    vultr = {"type": "vultr", "creds": {"type": "api_key", "api_key": "VULTR-KEY"}}
    runpod = {"type": "runpod", "creds": {"type": "api_key", "api_key": "RP-KEY"}}
    path = tmp_path / "config.yml"
    m = ServerConfigManager(path)
    _apply(m, path, {"projects": [{"name": "team", "backends": [vultr, runpod]}]})
    assert _backend_types("team") == ["runpod", "vultr"] and sorted(checks) == ["runpod", "vultr"]
    # the same file again: nothing is re-validated (no cloud round-trip per restart) or rewritten
    checks.clear()
    _apply(m, path, {"projects": [{"name": "team", "backends": [vultr, runpod]}]})
    assert checks == []
    # a changed credential is applied; the unchanged backend is still skipped
    vultr2 = {"type": "vultr", "creds": {"type": "api_key", "api_key": "VULTR-KEY-2"}}
    _apply(m, path, {"projects": [{"name": "team", "backends": [vultr2, runpod]}]})
    assert checks == ["vultr"]
    # runpod removed from the file -> deleted; an invalid aws entry and an unknown type are skipped
    bad = [{"type": "aws", "creds": {"type": "access_key"}}, {"type": "no-such-cloud"}]
    _apply(m, path, {"projects": [{"name": "team", "backends": [vultr2, *bad]}]})
    assert _backend_types("team") == ["vultr"]
    with session_scope() as s:
        project = s.query(ProjectModel).filter_by(name="team").one()
        (b,) = s.query(BackendModel).filter_by(project_id=project.id).all()
        assert json.loads(b.auth)["api_key"] == "VULTR-KEY-2"


def test_server_config_keeps_unlisted_backend_with_live_instances(db, tmp_path, keys):
    from dstack_amd.core.models.instances import InstanceStatus
    from dstack_amd.server.services import pools as pools_services
    from dstack_amd.server.services.config import ServerConfigManager

    vultr = {"type": "vultr", "creds": {"type": "api_key", "api_key": "VULTR-KEY"}}
    path = tmp_path / "config.yml"
    m = ServerConfigManager(path)
    _apply(m, path, {"projects": [{"name": "team", "backends": [vultr]}]})
    with session_scope() as s:
        project = s.query(ProjectModel).filter_by(name="team").one()
        pool = pools_services.get_or_create_default_pool(s, project)
        inst = pools_services.create_instance_model(s, project, pool, "vm-1", InstanceStatus.IDLE)
        inst.backend = "vultr"
    _apply(m, path, {"projects": [{"name": "team", "backends": []}]})
    assert _backend_types("team") == ["vultr"]  # logged and kept until its instance is gone


def test_server_starts_with_one_invalid_backend_in_config(db, tmp_path, keys, monkeypatch):
    """``init_server_state`` with a config.yml holding an invalid backend next to a valid one: the
    server starts and the valid backend is configured (the reference logs and continues)."""
    from dstack_amd.server import settings
    from dstack_amd.server.app import init_server_state

    path = tmp_path / "config.yml"
    path.write_text(yaml.safe_dump({"projects": [{"name": "main", "backends": [
        {"type": "aws", "creds": {"type": "access_key", "access_key": "AKIA"}},  # no secret_key
        {"type": "vultr", "creds": {"type": "api_key", "api_key": "VULTR-KEY"}}]}]}))
    monkeypatch.setattr(settings, "SERVER_CONFIG_FILE_PATH", str(path))
    monkeypatch.setattr(settings, "SERVER_CONFIG_DISABLED", False)
    assert init_server_state()
    assert _backend_types("main") == ["vultr"]
