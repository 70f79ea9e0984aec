"""Core models, client-side services and utilities, case by case against the reference's
``src/tests/_internal/{core,utils}`` and ``src/tests/api`` (mapping: ``docs/reference/test-parity.md``):
resource / GPU spec parsing and range intersection, mount points, unix users, termination-reason
mappings, GPU vendor inference, configuration rules, git remote URLs with ``~/.ssh/config``
aliases, log URL rewriting, SSH client capabilities and tunnel command lines, and the small
helpers (dates, memory quantities, chunks, URL joins, env booleans, relative paths)."""

from __future__ import annotations

import subprocess
from datetime import datetime, timedelta, timezone
from pathlib import Path, PurePath
from unittest import mock

import pytest
from pydantic import TypeAdapter, ValidationError

from dstack_amd.core.models.resources import AcceleratorVendor, ComputeCapability, GPUSpec, IntRange, Memory, MemoryRange


def P(tp, v):
    return TypeAdapter(tp).validate_python(v)


# ---- core/models/test_resources.py --------------------------------------------------------------
@pytest.mark.parametrize("v,expected", [("512MB", 0.5), ("16 Gb", 16.0), ("1 TB ", 1024.0), (1.5, 1.5), (1, 1.0)],
                         ids=["mb", "gb", "tb", "float", "int"])
def test_memory_units(v, expected):
    assert P(Memory, v) == expected


def test_memory_invalid():
    with pytest.raises(ValidationError):
        P(Memory, "1.5xb")


@pytest.mark.parametrize("v,expected", [("3.5", (3, 5)), (8.0, (8, 0)), ((7, 5), (7, 5))], ids=["str", "float", "tuple"])
def test_compute_capability_forms(v, expected):
    assert P(ComputeCapability, v) == expected


@pytest.mark.parametrize("v", ["3.5.1", "3.x"], ids=["invalid_len", "invalid_type"])
def test_compute_capability_invalid(v):
    with pytest.raises(ValidationError):
        P(ComputeCapability, v)


@pytest.mark.parametrize("v,expected", [(1, (1, 1)), ("1", (1, 1)), ("1..", (1, None)), ("..1", (None, 1)),
                                        ({"min": 1, "max": 3}, (1, 3))], ids=["int", "exact", "from", "to", "dict"])
def test_int_range_forms(v, expected):
    r = P(IntRange, v)
    assert (r.min, r.max) == expected and isinstance(str(r), str)


@pytest.mark.parametrize("v", ["..", "1...3", "3..1"], ids=["invalid_range", "typo", "unordered"])
def test_int_range_invalid(v):
    with pytest.raises(ValidationError):
        P(IntRange, v)


@pytest.mark.parametrize("v,expected", [("512MB", (0.5, 0.5)), ("512MB..", (0.5, None)), ("..1 TB", (None, 1024.0)),
                                        ("512..1 TB", (512.0, 1024.0)), ({"min": "512MB", "max": "1TB"}, (0.5, 1024.0))],
                         ids=["mb", "from", "to", "range", "dict"])
def test_memory_range_forms(v, expected):
    r = P(MemoryRange, v)
    assert (r.min, r.max) == expected


def test_memory_range_invalid():
    with pytest.raises(ValidationError):
        P(MemoryRange, "...")


@pytest.mark.parametrize("value,expected", [
    ("1", {"count": 1}),
    ("Nvidia", {"vendor": "nvidia"}),
    ("google:v3-64", {"vendor": "google", "name": ["v3-64"]}),
    ("tpu:v5p-1024", {"vendor": "google", "name": ["v5p-1024"]}),
    ("v5litepod-64:TPU", {"vendor": "google", "name": ["v5litepod-64"]}),
    ("MI300X:AMD", {"vendor": "amd", "name": ["MI300X"]}),
    ("A100", {"name": ["A100"]}),
    ("16GB", {"memory": "16GB"}),
    ("A10,A10G:2", {"name": ["A10", "A10G"], "count": 2}),
    ("16GB..32", {"memory": {"min": 16, "max": 32}}),
])
def test_gpu_spec_string_form(value, expected):
    assert P(GPUSpec, value) == P(GPUSpec, expected)


@pytest.mark.parametrize("value,expected", [(None, None), ("NVIDIA", "nvidia"), ("amd", "amd"), ("Google", "google"),
                                            ("tpu", "google"), ("TPU", "google"), (AcceleratorVendor.GOOGLE, "google")])
def test_gpu_spec_vendor_object_form(value, expected):
    assert P(GPUSpec, {"vendor": value}) == P(GPUSpec, {"vendor": expected})


def test_gpu_spec_tpu_prefix_stripped():
    assert P(GPUSpec, "tpu-v3-2048").name == ["v3-2048"]


@pytest.mark.parametrize("value,match", [("A100,:2", None), ("A100:", None), ("Nvidia:A100:2:AMD", "vendor conflict"),
                                         ("A100:2:3", "count conflict")],
                         ids=["empty_name", "empty_token", "vendor_conflict", "count_conflict"])
def test_gpu_spec_invalid(value, match):
    with pytest.raises(ValidationError, match=match):
        P(GPUSpec, value)


@pytest.mark.parametrize("r1,r2,expected", [
    ((1, 2), (3, 4), None), ((1, 2), (2, 3), (2, 2)), ((1, 2), (1, 2), (1, 2)), ((1, 3), (2, 4), (2, 3)),
    ((1, 4), (2, 3), (2, 3)), ((None, 1), (2, None), None), ((None, 1), (1, None), (1, 1)),
    ((None, 2), (1, None), (1, 2)), ((None, 1), (None, 2), (None, 1)), ((1, None), (2, None), (2, None)),
    ((1, None), (None, 2), (1, 2)),
])
def test_intersect_ranges(r1, r2, expected):
    a, b = IntRange(min=r1[0], max=r1[1]), IntRange(min=r2[0], max=r2[1])
    for x, y in ((a, b), (b, a)):
        got = x.intersect(y)
        assert (None if got is None else (got.min, got.max)) == expected


# ---- core/models/test_volumes.py ----------------------------------------------------------------
def test_volume_mount_point_parse_and_normalisation():
    from dstack_amd.core.models.volumes import VolumeMountPoint

    assert VolumeMountPoint.parse("my-vol:/path/./to///dir/") == VolumeMountPoint(name="my-vol", path="/path/to/dir")
    assert P(VolumeMountPoint, {"name": "my-vol", "path": "/path/./to///dir/"}) == \
        VolumeMountPoint(name="my-vol", path="/path/to/dir")


def test_instance_mount_point_parse_and_normalisation():
    from dstack_amd.core.models.volumes import InstanceMountPoint

    want = InstanceMountPoint(instance_path="/host/path", path="/run/path")
    assert InstanceMountPoint.parse("/host/.//path/:/run//./path") == want
    assert P(InstanceMountPoint, {"instance_path": "/host/.//path/", "path": "/run//./path"}) == want


@pytest.mark.parametrize("value", ["my-vol", "my-vol:/run:ro", "/path", "/host/path:/run/path:ro"])
def test_mount_point_invalid_format(value):
    from dstack_amd.core.models.volumes import parse_mount_point

    with pytest.raises(ValueError, match="invalid mount point format"):
        parse_mount_point(value)


@pytest.mark.parametrize("kind", ["volume", "instance_path", "instance_run_path"])
@pytest.mark.parametrize("bad,match", [("", "empty path"), ("rel/path", "path must be absolute"),
                                       ("/path/../to", r"\.\. are not allowed")])
def test_mount_point_path_validation(kind, bad, match):
    from dstack_amd.core.models.volumes import InstanceMountPoint, VolumeMountPoint

    if kind == "volume":
        cls, data = VolumeMountPoint, {"name": "vol", "path": bad}
    else:
        data = {"instance_path": "/instance_path", "path": "/run_path"}
        data["instance_path" if kind == "instance_path" else "path"] = bad
        cls = InstanceMountPoint
    with pytest.raises(ValidationError, match=match):
        P(cls, data)


def test_parse_mount_point_kinds():
    from dstack_amd.core.models.volumes import InstanceMountPoint, VolumeMountPoint, parse_mount_point

    assert parse_mount_point("my-vol:/path//to") == VolumeMountPoint(name="my-vol", path="/path/to")
    assert parse_mount_point("/host:/run/") == InstanceMountPoint(instance_path="/host", path="/run")
    for v in ["path/to:/run", "./path:/run", "path/:/run"]:
        with pytest.raises(ValidationError, match="path must be absolute"):
            parse_mount_point(v)


# ---- core/models/test_unix.py, test_runs.py, test_instances.py, test_configurations.py ----------
@pytest.mark.parametrize("value,expected", [
    ("0", {"uid": 0}), ("1000", {"uid": 1000}), ("debian", {"username": "debian"}), ("1000:2000", {"uid": 1000, "gid": 2000}),
    ("1000:wheel", {"uid": 1000, "groupname": "wheel"}), ("root:0", {"username": "root", "gid": 0}),
    ("admin:wheel", {"username": "admin", "groupname": "wheel"}),
])
def test_unix_user_parse(value, expected):
    from dstack_amd.core.models.unix import UnixUser

    assert UnixUser.parse(value) == UnixUser(**expected)


@pytest.mark.parametrize("value,match", [
    ("1000:1000:", "too many parts"), ("user:group:foo:bar", "too many parts"), ("", "empty user name or id"),
    (":group", "empty user name or id"), ("-1", "negative uid"), ("-1:group", "negative uid"),
    ("user:", "empty group name or id"), ("1000:-1000", "negative gid"),
])
def test_unix_user_parse_errors(value, match):
    from dstack_amd.core.models.unix import UnixUser

    with pytest.raises(ValueError, match=match):
        UnixUser.parse(value)


def test_termination_reasons_map_for_every_variant():
    from dstack_amd.core.models.runs import JobStatus, JobTerminationReason, RunStatus, RunTerminationReason

    for r in RunTerminationReason:
        assert isinstance(r.to_job_termination_reason(), JobTerminationReason)
        assert isinstance(r.to_status(), RunStatus)
    for j in JobTerminationReason:
        assert isinstance(j.to_status(), JobStatus)


@pytest.mark.parametrize("data,vendor,name", [
    ({"name": "T4", "memory_mib": 16}, AcceleratorVendor.NVIDIA, "T4"),
    ({"name": "tpu-v3", "memory_mib": 0}, AcceleratorVendor.GOOGLE, "v3"),
    ({"vendor": "AMD", "name": "MI300X", "memory_mib": 192}, AcceleratorVendor.AMD, "MI300X"),
    ({"name": "MI355X", "memory_mib": 288 * 1024}, AcceleratorVendor.AMD, "MI355X"),  # MI355X build: inferred
])
def test_gpu_vendor_inferred(data, vendor, name):
    from dstack_amd.core.models.instances import Gpu

    g = Gpu.model_validate(data)
    assert g.vendor == vendor and g.name == name


def test_service_replicas_range_needs_scaling():
    from dstack_amd.core.errors import ConfigurationError
    from dstack_amd.core.models.configurations import parse_run_configuration

    def conf(replicas, scaling=None):
        c = {"type": "service", "commands": ["python3 -m http.server"], "port": 8000, "replicas": replicas}
        return {**c, "scaling": scaling} if scaling else c

    for v, want in ((1, (1, 1)), ("2", (2, 2)), ("3..3", (3, 3))):
        r = parse_run_configuration(conf(v)).replicas
        assert (r.min, r.max) == want
    with pytest.raises((ConfigurationError, ValidationError), match="ensure to specify `scaling`"):
        parse_run_configuration(conf("0..10"))
    r = parse_run_configuration(conf("0..10", {"metric": "rps", "target": 10})).replicas
    assert (r.min, r.max) == (0, 10)
    with pytest.raises((ConfigurationError, ValidationError)):
        parse_run_configuration(conf("0..10", {"metric": "rpc", "target": 10}))


def test_registry_auth_hashable():
    from dstack_amd.core.models.common import RegistryAuth

    a, b = RegistryAuth(username="u", password="p"), RegistryAuth(username="u", password="p")
    assert hash(a) == hash(b) and len({a, b}) == 1


# ---- core/models/repos/test_remote.py -----------------------------------------------------------
def _cfg(d):
    return lambda host: d.get(host, {})


@pytest.mark.parametrize("url,cfg,https,ssh", [
    ("https://github.com/dstackai/dstack.git", {}, "https://github.com/dstackai/dstack.git",
     "ssh://git@github.com/dstackai/dstack.git"),
    ("https://github.com:8443/dstackai/dstack.git", {}, "https://github.com:8443/dstackai/dstack.git",
     "ssh://git@github.com/dstackai/dstack.git"),
    ("https://github.com:8443/dstackai/dstack.git",
     {"github.com": {"user": "test-user", "port": "2222", "hostname": "test.github.com"}},
     "https://github.com:8443/dstackai/dstack.git", "ssh://test-user@github.com:2222/dstackai/dstack.git"),
    ("test-user@test.example:a/b/c.git", {}, "https://test.example/a/b/c.git", "ssh://test-user@test.example/a/b/c.git"),
    ("test-user@test.example:a/b/c.git",
     {"test.example": {"user": "test-user-2", "port": "2222", "hostname": "test2.example"}},
     "https://test2.example/a/b/c.git", "ssh://test-user@test2.example:2222/a/b/c.git"),
    ("ssh://test/repo.git", {"test": {"user": "test-user", "port": "2222", "hostname": "test.example"}},
     "https://test.example/repo.git", "ssh://test-user@test.example:2222/repo.git"),
], ids=["https", "https_port", "https_ssh_config", "scp", "scp_ssh_config", "ssh_url_ssh_config"])
def test_git_repo_url(url, cfg, https, ssh):
    from dstack_amd.core.models.repos import GitRepoURL

    u = GitRepoURL.parse(url, get_ssh_config=_cfg(cfg))
    assert u.as_https() == https and u.as_ssh() == ssh


@pytest.mark.parametrize("url", ["ftp://test.example/group/repo.git", "garbage"])
def test_git_repo_url_rejects(url):
    from dstack_amd.core.models.repos import GitRepoURL, RepoError

    with pytest.raises(RepoError):
        GitRepoURL.parse(url, get_ssh_config=_cfg({}))


def test_git_repo_url_oauth_token():
    from dstack_amd.core.models.repos import GitRepoURL

    u = GitRepoURL.parse("https://github.com/dstackai/dstack.git", get_ssh_config=_cfg({}))
    assert u.as_https("secret-token") == "https://anything:secret-token@github.com/dstackai/dstack.git"


def test_ssh_config_lookup(tmp_path):
    from dstack_amd.utils.ssh import get_ssh_config

    p = tmp_path / "config"
    p.write_text("User default-user\nHost gpu-*\n  HostName 10.0.0.5\n  Port 2222\nHost !gpu-x *\n  User other\n")
    assert get_ssh_config("gpu-1", str(p)) == {"user": "default-user", "hostname": "10.0.0.5", "port": "2222"}
    assert get_ssh_config("box", str(p)) == {"user": "default-user"}
    assert get_ssh_config("x", str(tmp_path / "missing")) == {}


# ---- core/services/test_logs.py: URL rewriting of job logs --------------------------------------
def _R(ports, apps=(), host="127.0.0.1", secure=False, **kw):
    from dstack_amd.core.models.runs import AppSpec
    from dstack_amd.core.services.logs import URLReplacer

    return URLReplacer(ports=ports, app_specs=[AppSpec(**a) for a in apps], hostname=host, secure=secure, **kw)


@pytest.mark.parametrize("rep,src,want", [
    (dict(ports={}, apps=[{"port": 3001, "app_name": "q"}]), b"http://0.0.0.0:3001/qwerty", b"http://0.0.0.0:3001/qwerty"),
    (dict(ports={3001: 3001}, apps=[{"port": 3001, "app_name": "q"}], host="host.name"),
     b"http://0.0.0.0:3001/qwerty", b"http://host.name:3001/qwerty"),
    (dict(ports={4000: 5000, 3001: 5501}, apps=[{"port": 3001, "app_name": "q"}]),
     b"http://0.0.0.0:3001/qwerty", b"http://127.0.0.1:5501/qwerty"),
    (dict(ports={4000: 5000, 3001: 5501}, apps=[{"port": 3001, "app_name": "q", "url_query_params": {"q": "foobar"}}]),
     b"http://0.0.0.0:3001/qwerty", b"http://127.0.0.1:5501/qwerty?q=foobar"),
    (dict(ports={4000: 5000, 3001: 5501}, apps=[{"port": 3001, "app_name": "q"}]),
     b"http://0.0.0.0:3001/qwerty and http://0.0.0.0:3001/foobar",
     b"http://127.0.0.1:5501/qwerty and http://127.0.0.1:5501/foobar"),
    (dict(ports={4000: 5000, 3001: 5501, 3002: 5502}, apps=[{"port": 3001, "app_name": "a"}, {"port": 3002, "app_name": "b"}]),
     b"http://0.0.0.0:3001/qwerty and http://0.0.0.0:3002/foobar",
     b"http://127.0.0.1:5501/qwerty and http://127.0.0.1:5502/foobar"),
    (dict(ports={4000: 5000, 3001: 3002, 3002: 3003, 3003: 3001}),
     b"http://0.0.0.0:3001/a and http://0.0.0.0:3002/b and http://0.0.0.0:3003/c",
     b"http://127.0.0.1:3002/a and http://127.0.0.1:3003/b and http://127.0.0.1:3001/c"),
    (dict(ports={3615: 53615}, apps=[{"port": 3615, "app_name": "fastapi"}]),
     b"\x1b[32mINFO\x1b[0m:     Uvicorn running on \x1b[1mhttp://0.0.0.0:3615\x1b[0m (Press CTRL+C to quit)",
     b"\x1b[32mINFO\x1b[0m:     Uvicorn running on \x1b[1mhttp://127.0.0.1:53615\x1b[0m (Press CTRL+C to quit)"),
    (dict(ports={3001: 3002}, ip_address="1.2.3.4"), b"http://1.2.3.4:3001/qwerty", b"http://127.0.0.1:3002/qwerty"),
], ids=["empty_mapping", "hostname", "unique_mapping", "query_params", "same_url", "different_urls", "circular",
        "fastapi", "ip_address"])
def test_task_url_replacer(rep, src, want):
    rep = dict(rep)
    assert _R(rep.pop("ports"), rep.pop("apps", ()), **rep)(src) == want


def test_service_url_replacer_ports_and_default_ports():
    assert _R({8000: 8080}, host="1.2.3.4")(b"http://0.0.0.0:8000") == b"http://1.2.3.4:8080"
    assert _R({8000: 80}, host="1.2.3.4")(b"http://0.0.0.0:8000/qwerty") == b"http://1.2.3.4/qwerty"
    assert _R({8000: 443}, host="secure.host.com", secure=True)(b"http://0.0.0.0:8000/qwerty") == \
        b"https://secure.host.com/qwerty"


@pytest.mark.parametrize("in_path,out_path", [
    ("", "/proxy/services/main/service/"), ("/", "/proxy/services/main/service/"),
    ("/a/b/c", "/proxy/services/main/service/a/b/c"), ("/proxy/services/main/service", "/proxy/services/main/service"),
    ("/proxy/services/main/service/", "/proxy/services/main/service/"),
    ("/proxy/services/main/service/a/b/c", "/proxy/services/main/service/a/b/c"),
])
def test_service_url_replacer_adds_prefix_unless_present(in_path, out_path):
    r = _R({8888: 3000}, host="0.0.0.0", path_prefix="/proxy/services/main/service/")
    assert r(f"http://0.0.0.0:8888{in_path}".encode()) == f"http://0.0.0.0:3000{out_path}".encode()


# ---- core/services/ssh/test_client.py, test_tunnel.py ------------------------------------------
@pytest.mark.parametrize("raw,version,vt,win,ctrl,mux,bg,host_win", [
    ("OpenSSH_9.7, LibreSSL 3.9.0", "9.7", (9, 7), False, True, True, True, False),
    ("OpenSSH_9.2p1 Debian-2+deb12u3, OpenSSL 3.0.13 30 Jan 2024", "9.2p1", (9, 2), False, True, True, True, False),
    ("OpenSSH_9.7p1, LibreSSL 3.3.6", "9.7p1", (9, 7), False, True, True, True, False),
    ("OpenSSH_9.8p1, OpenSSL 3.2.2 4 Jun 2024", "9.8p1", (9, 8), False, True, False, True, True),
    ("OpenSSH_for_Windows_8.6p1, LibreSSL 3.4.3", "8.6p1", (8, 6), True, False, False, False, True),
], ids=["openbsd", "linux", "macos", "windows_msys2", "windows_for_windows"])
def test_ssh_client_info(raw, version, vt, win, ctrl, mux, bg, host_win):
    from dstack_amd.utils.ssh import SSHClientInfo

    i = SSHClientInfo.from_raw_version(raw, Path("/usr/bin/ssh"), windows_host=host_win)
    assert (i.version, i.version_tuple, i.for_windows) == (version, vt, win)
    assert (i.supports_control_socket, i.supports_multiplexing, i.supports_background_mode) == (ctrl, mux, bg)


def _tunnel(**kw):
    from dstack_amd.core.services.ssh.tunnel import SSHTarget, SSHTunnel

    target = kw.pop("target", SSHTarget("my-server", "ubuntu", kw.pop("port", 22), kw.pop("proxy", None)))
    return SSHTunnel(target, ssh_binary="/usr/bin/ssh", **kw)


def test_tunnel_open_command_basic():
    t = _tunnel(identity_file="/home/user/.ssh/id_rsa", control_sock_path="/tmp/control.sock",
                options={"Opt1": "opt1", "Opt2": "opt2"}, ssh_config_path="/home/user/.ssh/config", port=10022)
    assert " ".join(t.open_command()) == (
        f"/usr/bin/ssh -F /home/user/.ssh/config -i /home/user/.ssh/id_rsa -E {t.temp_dir.name}/tunnel.log -N -f"
        " -o ControlMaster=auto -S /tmp/control.sock -p 10022 -o Opt1=opt1 -o Opt2=opt2 ubuntu@my-server")


def test_tunnel_temp_identity_and_control_socket():
    t = _tunnel(identity_content="my private key", options={})
    d = t.temp_dir.name
    assert " ".join(t.open_command()) == (f"/usr/bin/ssh -F none -i {d}/identity -E {d}/tunnel.log -N -f"
                                          f" -o ControlMaster=auto -S {d}/control.sock ubuntu@my-server")
    assert (Path(d) / "identity").read_text() == "my private key"
    assert (Path(d) / "identity").stat().st_mode & 0o077 == 0


def test_tunnel_open_command_with_proxy():
    from dstack_amd.core.services.ssh.tunnel import SSHTarget

    t = _tunnel(identity_file="/home/user/.ssh/id_rsa", control_sock_path="/tmp/control.sock", options={},
                proxy=SSHTarget("proxy", "test", 10022))
    cmd = t.open_command()
    assert cmd[cmd.index("ProxyCommand=/usr/bin/ssh -i /home/user/.ssh/id_rsa -W %h:%p -o StrictHostKeyChecking=no"
                         " -o UserKnownHostsFile=/dev/null -p 10022 test@proxy")] and cmd[-1] == "ubuntu@my-server"


def test_tunnel_open_command_with_forwarding():
    from dstack_amd.core.services.ssh.tunnel import IPSocket, SocketPair, UnixSocket

    t = _tunnel(identity_file="/k", control_sock_path="/tmp/control.sock", options={},
                forwarded_sockets=[SocketPair(UnixSocket("/tmp/80"), IPSocket("localhost", 80)),
                                   SocketPair(IPSocket("127.0.0.1", 8000), IPSocket("::1", 80))],
                reverse_forwarded_sockets=[SocketPair(UnixSocket("/tmp/local"), UnixSocket("/tmp/remote")),
                                           SocketPair(IPSocket("test.local", 80), IPSocket("localhost", 8000))])
    assert " ".join(t.open_command()).endswith(
        "-S /tmp/control.sock -L /tmp/80:localhost:80 -L 127.0.0.1:8000:[::1]:80 -R /tmp/remote:/tmp/local"
        " -R localhost:8000:test.local:80 ubuntu@my-server")


def test_tunnel_check_close_exec_commands():
    t = _tunnel(identity_file="/k", control_sock_path="/tmp/control.sock")
    assert t.check_command() == ["/usr/bin/ssh", "-S", "/tmp/control.sock", "-O", "check", "ubuntu@my-server"]
    assert t.close_command() == ["/usr/bin/ssh", "-S", "/tmp/control.sock", "-O", "exit", "ubuntu@my-server"]
    assert t.exec_command() == ["/usr/bin/ssh", "-S", "/tmp/control.sock", "ubuntu@my-server"]


def test_ports_to_forwarded_sockets():
    from dstack_amd.core.services.ssh.tunnel import IPSocket, SocketPair, ports_to_forwarded_sockets

    assert ports_to_forwarded_sockets({80: 8000, 22: 2200}, bind_local="::1") == [
        SocketPair(IPSocket("::1", 8000), IPSocket("localhost", 80)),
        SocketPair(IPSocket("::1", 2200), IPSocket("localhost", 22))]


# ---- utils/test_common.py -----------------------------------------------------------------------
def test_local_time():
    from dstack_amd.utils.common import local_time

    assert local_time(datetime.fromisoformat("1970-01-01T12:34")) == "12:34"
    assert local_time(datetime.fromisoformat("2024-12-01T01:02:03")) == "01:02"


_NOW = datetime(2023, 10, 4, 12, 0, tzinfo=timezone.utc)


@pytest.mark.parametrize("delta,want", [
    (timedelta(0), "now"), (timedelta(seconds=30), "30 sec ago"), (timedelta(minutes=1), "1 min ago"),
    (timedelta(minutes=45), "45 mins ago"), (timedelta(hours=1), "1 hour ago"), (timedelta(hours=5), "5 hours ago"),
    (timedelta(days=1), "yesterday"), (timedelta(days=5), "5 days ago"), (timedelta(days=21), "3 weeks ago"),
    (timedelta(days=90), "3 months ago"), (timedelta(days=400), "1 year ago"), (-timedelta(hours=1), ""),
], ids=["now", "seconds", "one_minute", "minutes", "one_hour", "hours", "yesterday", "days", "weeks", "months",
        "years", "future"])
def test_pretty_date(delta, want):
    from dstack_amd.utils.common import pretty_date

    assert pretty_date(_NOW - delta, now=_NOW) == want


@pytest.mark.parametrize("memory,units,want", [("1024Ki", "M", 1), ("512Ki", "M", 0.5), ("2Gi", "M", 2048),
                                               ("1024Ki", "K", 1024)])
def test_parse_memory(memory, units, want):
    from dstack_amd.utils.common import parse_memory

    assert parse_memory(memory, as_untis=units) == want


@pytest.mark.parametrize("it,n,want", [
    ([1, 2, 3, 4], 2, [[1, 2], [3, 4]]), ([1, 2, 3], 2, [[1, 2], [3]]), ([1, 2], 2, [[1, 2]]), ([1], 2, [[1]]),
    ([], 2, []), ({"a": 1, "b": 2, "c": 3}, 2, [["a", "b"], ["c"]]), ((x for x in range(5)), 3, [[0, 1, 2], [3, 4]]),
])
def test_split_chunks(it, n, want):
    from dstack_amd.utils.common import split_chunks

    assert list(split_chunks(it, n)) == want


@pytest.mark.parametrize("n", [0, -1])
def test_split_chunks_rejects_bad_size(n):
    from dstack_amd.utils.common import split_chunks

    with pytest.raises(ValueError):
        list(split_chunks([1, 2, 3], n))


@pytest.mark.parametrize("a,b,want", [("/a/b", "c/d", "/a/b/c/d"), ("/a/b/", "/c/d", "/a/b/c/d"),
                                      ("/a/b//", "//c/d", "/a/b///c/d"), ("/a", "", "/a"), ("/a", "/", "/a/"),
                                      ("", "a", "/a"), ("/", "a", "/a"), ("", "", "")])
def test_concat_url_path(a, b, want):
    from dstack_amd.utils.common import concat_url_path

    assert concat_url_path(a, b) == want
    assert concat_url_path(a.encode(), b.encode()) == want.encode()


@pytest.mark.parametrize("server,proxy,want", [
    ("http://localhost:3000", "https://gateway.mycompany.example/", "https://gateway.mycompany.example/"),
    ("https://dstack.mycompany.example/", "http://gateway.mycompany.example/some/path", "http://gateway.mycompany.example/some/path"),
    ("http://localhost:3000", "/proxy/services/main/service/", "http://localhost:3000/proxy/services/main/service/"),
    ("http://localhost:3000/", "/proxy/models/main", "http://localhost:3000/proxy/models/main"),
    ("https://dstack.mycompany.example/some/prefix", "/proxy/models/main",
     "https://dstack.mycompany.example/some/prefix/proxy/models/main"),
])
def test_make_proxy_url(server, proxy, want):
    from dstack_amd.utils.common import make_proxy_url

    assert make_proxy_url(server, proxy) == want


# ---- utils/test_env.py, test_gpu.py, test_network.py, test_path.py, test_ssh.py ------------------
@pytest.mark.parametrize("value,want", [("0", False), ("1", True), ("true", True), ("True", True), ("FALSE", False),
                                        ("off", False), ("ON", True)])
def test_get_bool_set(monkeypatch, value, want):
    from dstack_amd.utils.env import get_bool

    monkeypatch.setenv("VAR", value)
    assert get_bool("VAR") is want


@pytest.mark.parametrize("default", [None, False, True])
def test_get_bool_unset(monkeypatch, default):
    from dstack_amd.utils.env import get_bool

    monkeypatch.delenv("VAR", raising=False)
    assert get_bool("VAR") is False if default is None else get_bool("VAR", default) is default


@pytest.mark.parametrize("value", ["", "2", "foo"])
def test_get_bool_error(monkeypatch, value):
    from dstack_amd.utils.env import get_bool

    monkeypatch.setenv("VAR", value)
    with pytest.raises(ValueError, match=f"VAR={value}"):
        get_bool("VAR")


@pytest.mark.parametrize("raw,want", [
    ("NVIDIA GeForce RTX 4060 Ti", "RTX4060Ti"), ("NVIDIA GeForce RTX 4060", "RTX4060"),
    ("NVIDIA RTX 4000 Ada Generation", "RTX4000Ada"), ("NVIDIA L4", "L4"), ("NVIDIA GH200 120GB", "GH200"),
    ("NVIDIA A100-SXM4-80GB", "A100"), ("NVIDIA A10G", "A10G"), ("NVIDIA L40S", "L40S"), ("NVIDIA H100 NVL", "H100NVL"),
    ("NVIDIA H100 80GB HBM3", "H100"), ("Tesla T4", "T4"),
])
def test_convert_nvidia_gpu_name(raw, want):
    from dstack_amd.core.models.gpus import convert_nvidia_gpu_name

    assert convert_nvidia_gpu_name(raw) == want


@pytest.mark.parametrize("raw,want", [
    ("MI300X-O", "MI300X"), ("Instinct MI210", "MI210"), ("AMD INSTINCT MI250 (MCM) OAM AC MBA", "MI250"),
    ("MI300A", "MI300A"), ("Instinct MI325X", "MI325X"), ("AMD Radeon PRO W7900", "AMD Radeon PRO W7900"),
    ("AMD Instinct MI355 OAM", "MI355X"),  # what amd-smi reports for an MI355X
])
def test_convert_amd_gpu_name(raw, want):
    from dstack_amd.core.models.gpus import convert_amd_gpu_name

    assert convert_amd_gpu_name(raw) == want


@pytest.mark.parametrize("raw,want", [("HL-225", "Gaudi2"), ("HL-225B", "Gaudi2"), ("HL-325L", "Gaudi3"),
                                      ("HL-338", "Gaudi3"), ("HL-1000", "HL-1000")])
def test_convert_intel_accelerator_name(raw, want):
    from dstack_amd.core.models.gpus import convert_intel_accelerator_name

    assert convert_intel_accelerator_name(raw) == want


@pytest.mark.parametrize("network,addrs,want", [
    (None, [], None), ("192.168.1.0/24", ["192.168.1.23"], "192.168.1.23"), ("192.168.1.1/32", ["192.168.1.23"], None),
    ("192.168.1.0/24", [], None), ("192.168.1.0/24", ["fe80::8d91:ba6b:b24d:9b41%4"], None),
], ids=["none", "regular", "miss_network", "no_ip", "ipv6"])
def test_get_ip_from_network(network, addrs, want):
    from dstack_amd.utils.common import get_ip_from_network

    assert get_ip_from_network(network, addrs) == want


def test_get_ip_from_network_any_ip():
    from dstack_amd.utils.common import get_ip_from_network

    addrs = ["192.168.1.23", "10.1.0.0"]
    assert get_ip_from_network(None, addrs) in addrs


def test_resolve_relative_path():
    from dstack_amd.utils.path import resolve_relative_path

    with pytest.raises(ValueError):
        resolve_relative_path("/tmp")
    with pytest.raises(ValueError):
        resolve_relative_path("repo/../..")
    assert resolve_relative_path("repo/./../repo2") == PurePath("repo2")


@pytest.mark.parametrize("stdout,stderr,want", [
    ("", "OpenSSH_8.6p1, LibreSSL 3.3.6", True), ("", "OpenSSH_8.2p1, LibreSSL 3.2.3", False),
    ("OpenSSH_for_Windows_8.7p1, LibreSSL 3.2.3", "", True), ("OpenSSH_for_Windows_8.1p1, LibreSSL 3.2.3", "", False),
], ids=["above_8_4", "below_8_4", "windows_above", "windows_below"])
def test_check_required_ssh_version(stdout, stderr, want):
    from dstack_amd.utils.ssh import check_required_ssh_version

    with mock.patch("subprocess.run", return_value=mock.MagicMock(returncode=0, stdout=stdout, stderr=stderr)):
        assert check_required_ssh_version() is want


def test_check_required_ssh_version_subprocess_error():
    from dstack_amd.utils.ssh import check_required_ssh_version

    with mock.patch("subprocess.run", side_effect=subprocess.CalledProcessError(1, "ssh -V")):
        assert check_required_ssh_version() is False
