"""Reference cases outside the server suite's main groups: ``server/utils/test_{common,routers}.py``,
``server/test_app.py``, ``api/test_utils.py`` and ``cli/commands/test_dstack.py``."""

from __future__ import annotations

from pathlib import Path

import pytest

from dstack_amd.server.utils.common import ajoin_byte_stream_checked, join_byte_stream_checked
from dstack_amd.server.utils.routers import check_client_server_compatibility


# ---- server/utils/test_common.py --------------------------------------------------------------------
@pytest.mark.parametrize("stream,max_size,result", [
    ([b"12", b"34", b"56"], 7, b"123456"), ([b"12", b"34", b"56"], 6, b"123456"),
    ([b"12", b"34", b"56"], 5, None), ([b"12", b"34", b"56"], 0, None), ([], 0, b"")])
def test_join_byte_stream_checked(stream, max_size, result):
    assert join_byte_stream_checked(iter(stream), max_size) == result


@pytest.mark.parametrize("stream,max_size", [([b"12", b"34", b"56"], 5), ([b"12", b"34", b"56"], 0)])
def test_join_byte_stream_checked_stops_iteration_when_limit_reached(stream, max_size):
    def gen():
        yield from stream
        raise RuntimeError("Stream end reached, but next value was requested")

    assert join_byte_stream_checked(gen(), max_size) is None


def test_ajoin_byte_stream_checked():
    import asyncio

    async def agen(chunks):
        for c in chunks:
            yield c
        raise RuntimeError("read past the limit")

    assert asyncio.run(ajoin_byte_stream_checked(agen([b"ab", b"cd", b"ef"]), 3)) is None


def test_code_upload_over_the_limit_is_refused_without_reading_it_all(client, monkeypatch):
    from dstack_amd.server.routers import core

    monkeypatch.setattr(core, "CODE_UPLOAD_LIMIT", 1000)
    r = client.post("/api/project/main/repos/upload_code?repo_id=r", content=b"x" * 100_000)
    assert r.status_code == 400 and "exceeds" in r.json()["detail"][0]["msg"]


def test_registry_config_blob_is_read_up_to_the_cap():
    import httpx

    from dstack_amd.core.errors import DockerRegistryError
    from dstack_amd.server.services import docker as docker_mod

    manifest = {"schemaVersion": 2, "mediaType": "application/vnd.oci.image.manifest.v1+json",
                "config": {"mediaType": "application/vnd.oci.image.config.v1+json", "digest": "sha256:c", "size": 1},
                "layers": []}
    big = b"{" + b" " * (docker_mod.MAX_CONFIG_OBJECT_SIZE + 10) + b"}"

    def handler(req):
        if "/manifests/" in req.url.path:
            return httpx.Response(200, json=manifest)
        return httpx.Response(200, content=big)

    rc = docker_mod.RegistryClient(httpx.Client(transport=httpx.MockTransport(handler)))
    with pytest.raises(DockerRegistryError, match="size limit"):
        rc.get_image_config("rocm/pytorch:latest")


# ---- server/utils/test_routers.py -------------------------------------------------------------------
@pytest.mark.parametrize("client_version", ["12.12.12", None])
def test_compat_none_if_server_version_is_none(client_version):
    assert check_client_server_compatibility(client_version, None) is None


@pytest.mark.parametrize("client_version,server_version", [
    ("0.12.4", "0.12.4"), ("0.12.4", "0.12.5"), ("0.12.4", "0.13.0"), ("0.12.4", "1.12.0"), ("0.12.4", "0.12.5rc1"),
    ("1.0.5", "1.0.6"), ("1.0.7", "1.0.6")])  # a newer patch release of the client is compatible too
def test_compat_none_if_compatible(client_version, server_version):
    assert check_client_server_compatibility(client_version, server_version) is None


@pytest.mark.parametrize("client_version,server_version", [("0.13.0", "0.12.4"), ("1.12.0", "0.12.0")])
def test_compat_error_if_client_version_larger(client_version, server_version):
    assert "incompatible" in check_client_server_compatibility(client_version, server_version)


@pytest.mark.parametrize("server_version", [None, "0.1.12"])
def test_compat_none_if_client_version_is_latest(server_version):
    assert check_client_server_compatibility("latest", server_version) is None


def test_compat_bad_version_and_server_middleware(client, monkeypatch):
    from dstack_amd.server import app as app_mod

    assert check_client_server_compatibility("not a version", "0.1.0") == "Bad API version specified"
    monkeypatch.setattr(app_mod, "__version__", "0.1.0")
    assert client.post("/api/server/get_info", headers={"X-API-VERSION": "0.1.9"}).status_code == 200
    r = client.post("/api/server/get_info", headers={"X-API-VERSION": "0.2.0"})
    assert r.status_code == 400 and "incompatible" in r.text
    assert client.post("/api/server/get_info", headers={"X-API-VERSION": "latest"}).status_code == 200


# ---- server/test_app.py ------------------------------------------------------------------------------
def test_index_returns_html(client):
    r = client.get("/")
    assert r.status_code == 200 and r.content.lower().startswith(b"<!doctype html>")


# ---- api/test_utils.py ----------------------------------------------------------------------------------
def test_load_profile_empty_when_no_profiles(monkeypatch, tmp_path):
    from dstack_amd.api.utils import load_profile

    monkeypatch.setenv("DSTACK_DIR", str(tmp_path / "home" / ".dstack"))
    p = load_profile(tmp_path / "repo", profile_name=None)
    assert p.name == "default" and p.backends is None


def test_load_profile_repo_then_global_then_error(monkeypatch, tmp_path):
    from dstack_amd.api.utils import load_profile
    from dstack_amd.core.errors import ConfigurationError

    home = tmp_path / "home" / ".dstack"
    home.mkdir(parents=True)
    monkeypatch.setenv("DSTACK_DIR", str(home))
    (home / "profiles.yml").write_text("profiles:\n- name: g\n  default: true\n  max_price: 2\n- name: other\n")
    repo = tmp_path / "repo"
    (repo / ".dstack").mkdir(parents=True)
    (repo / ".dstack" / "profiles.yaml").write_text("profiles:\n- name: r\n  max_price: 1\n")
    assert load_profile(repo, None).name == "g"  # the repo file marks no default: the global one is used
    assert load_profile(repo, "r").max_price == 1 and load_profile(repo, "other").name == "other"
    with pytest.raises(ConfigurationError, match="No such profile: nope"):
        load_profile(repo, "nope")


def test_load_configuration(tmp_path):
    from dstack_amd.api.utils import load_configuration
    from dstack_amd.core.errors import ConfigurationError

    (tmp_path / "sub").mkdir()
    (tmp_path / "sub" / ".dstack.yml").write_text("type: task\ncommands: [whoami]\n")
    path, conf = load_configuration(tmp_path, "sub")
    assert path == str(Path("sub") / ".dstack.yml") and conf.type == "task"
    with pytest.raises(ConfigurationError, match="outside the repo"):
        load_configuration(tmp_path / "sub", configuration_file="../x.yml")


# ---- cli/commands/test_dstack.py ---------------------------------------------------------------------------
def test_cli_prints_help_and_exits_with_0(capsys):
    from dstack_amd.cli.main import main

    assert main([]) == 0
    assert capsys.readouterr().out.startswith("usage: dstack [-h] [-v] COMMAND ...")
