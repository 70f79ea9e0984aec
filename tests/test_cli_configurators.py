"""CLI overrides applied by ``dstack apply`` (reference: ``src/tests/_internal/cli/services/
configurators/test_{run,profile,fleet}.py`` and ``cli/commands/test_config.py``): ``-e``/``-p``
merging, port conflicts, ``registry_auth`` interpolation, GPU vendor inference against the ROCm
default image, profile flags, and ``dstack config`` writing ``~/.dstack/config.yml``."""

from __future__ import annotations

import argparse

import pytest
import yaml

from dstack_amd.cli.configurators import (
    FleetConfigurator,
    RunConfigurator,
    apply_profile_args,
    register_profile_args,
    validate_gpu_vendor_and_image,
)
from dstack_amd.core.errors import ConfigurationError
from dstack_amd.core.models.configurations import PortMapping, TaskConfiguration
from dstack_amd.core.models.profiles import Profile, SpotPolicy


def _run_args(conf, argv):
    parser = argparse.ArgumentParser()
    RunConfigurator.register_args(parser)
    conf = conf.model_copy(deep=True)
    args, _ = parser.parse_known_args(argv)
    RunConfigurator.apply_args(conf, args)
    return conf


def _task(**kw):
    return TaskConfiguration.model_validate({"type": "task", "commands": ["whoami"], **kw})


# ---- run configurator ---------------------------------------------------------------------------
def test_env_args_add_and_override():
    conf = _run_args(_task(env={"A": "0"}), ["-e", "A=1", "--env", "B=2"])
    assert dict(conf.env) == {"A": "1", "B": "2"}


def test_env_arg_from_local_environment(monkeypatch):
    monkeypatch.setenv("FROM_ENV", "2")
    assert dict(_run_args(_task(), ["-e", "FROM_ENV"]).env) == {"FROM_ENV": "2"}
    monkeypatch.delenv("FROM_ENV")
    with pytest.raises(ConfigurationError, match="FROM_ENV is not set"):
        _run_args(_task(), ["-e", "FROM_ENV"])


def test_port_args():
    conf = _run_args(_task(), ["-p", "80", "--port", "8080"])
    assert conf.ports == [PortMapping(local_port=80, container_port=80),
                          PortMapping(local_port=8080, container_port=8080)]


def test_port_args_replace_same_container_port():
    conf = _run_args(_task(ports=["80"]), ["-p", "8000:80", "--port", "8001:8000"])
    assert conf.ports == [PortMapping(local_port=8000, container_port=80),
                          PortMapping(local_port=8001, container_port=8000)]


def test_any_local_port():
    conf = _run_args(_task(ports=["8000"]), ["-p", "*:8000"])
    assert conf.ports == [PortMapping(local_port=None, container_port=8000)]


@pytest.mark.parametrize("ports,argv", [([], ["-p", "8000:80", "--port", "8001:80"]),  # container port twice
                                        (["3000"], ["-p", "3000:4000"])])  # local port twice
def test_port_conflicts(ports, argv):
    with pytest.raises(ConfigurationError):
        _run_args(_task(ports=ports), argv)


def test_registry_auth_interpolates_env():
    conf = _run_args(_task(image="registry.example/img", env={"REG_USER": "u", "REG_PASS": "p"},
                           registry_auth={"username": "${{ env.REG_USER }}", "password": "${{ env.REG_PASS }}"}), [])
    assert (conf.registry_auth.username, conf.registry_auth.password) == ("u", "p")
    with pytest.raises(ConfigurationError, match="env.MISSING"):
        _run_args(_task(image="x", registry_auth={"username": "u", "password": "${{ env.MISSING }}"}), [])


def test_gpu_and_disk_args():
    conf = _run_args(_task(), ["--gpu", "MI355X:8", "--disk", "500GB.."])
    assert conf.resources.gpu.name == ["MI355X"] and conf.resources.gpu.count.min == 8
    assert conf.resources.gpu.vendor.value == "amd"
    assert conf.resources.disk.size.min == 500


# ---- GPU vendor inference vs the ROCm default image -----------------------------------------------
def _conf(gpu=None, image=None):
    d = {"type": "task", "commands": ["x"]}
    if gpu is not None:
        d["resources"] = {"gpu": gpu}
    if image is not None:
        d["image"] = image
    return TaskConfiguration.model_validate(d)


@pytest.mark.parametrize("gpu,vendor", [("MI355X", "amd"), ("mi300x", "amd"), ("MI300x:8", "amd"),
                                        ("amd", "amd"), ("nvidia", "nvidia"), ("a40,l40", "nvidia"),
                                        ("tpu", "google"), ("V3-64", "google")])
def test_vendor_declared_or_inferred(gpu, vendor):
    assert _conf(gpu, image="any").resources.gpu.vendor.value == vendor


@pytest.mark.parametrize("gpu", ["foo", "foo,bar", "A1000,v4", "v3-64,foo", "A1000,mi300x", "foo,MI300X"])
def test_vendor_not_inferred_from_mixed_or_unknown_names(gpu):
    conf = _conf(gpu)
    assert conf.resources.gpu.vendor is None
    validate_gpu_vendor_and_image(conf)  # unknown vendor: no image needed


@pytest.mark.parametrize("gpu", [None, "0", "MI355X:8", "amd", "mi300x"])
def test_amd_or_no_gpu_runs_on_default_image(gpu):
    validate_gpu_vendor_and_image(_conf(gpu))


@pytest.mark.parametrize("gpu", ["nvidia", "H100:8", "a40,l40", "tpu"])
def test_non_amd_gpu_requires_image(gpu):
    with pytest.raises(ConfigurationError, match="`image` is required"):
        validate_gpu_vendor_and_image(_conf(gpu))
    validate_gpu_vendor_and_image(_conf(gpu, image="my/cuda:12"))


# ---- profile flags ------------------------------------------------------------------------------
def _profile_args(argv):
    parser = argparse.ArgumentParser()
    register_profile_args(parser)
    prof = Profile(name="test")
    args = parser.parse_args(argv)
    apply_profile_args(args, prof)
    return prof, args


def test_profile_args_empty_and_name():
    prof, args = _profile_args(["--profile", "other"])
    assert prof.model_dump() == Profile(name="test").model_dump() and args.profile == "other"


def test_profile_args_values():
    prof, _ = _profile_args(["--max-price", "0.5", "--max-duration", "1h", "-b", "local", "--backend", "aws",
                             "--spot"])
    assert prof.max_price == 0.5 and prof.backends == ["local", "aws"]
    assert prof.spot_policy == SpotPolicy.SPOT
    assert prof.model_dump()["max_duration"] in (3600, "1h")
    assert _profile_args(["--on-demand"])[0].spot_policy == SpotPolicy.ONDEMAND


def test_profile_retry_flags():
    assert _profile_args(["--no-retry"])[0].retry is False
    prof = _profile_args(["--retry-duration", "1h"])[0]
    retry = prof.model_dump()["retry"]
    assert retry and retry["duration"] in (3600, "1h")
    assert _profile_args(["--retry"])[0].model_dump()["retry"]


# ---- fleet configurator ------------------------------------------------------------------------------
def _fleet_args(conf, argv):
    parser = argparse.ArgumentParser()
    FleetConfigurator.register_args(parser)
    args, _ = parser.parse_known_args(argv)
    conf = conf.model_copy(deep=True)
    FleetConfigurator.apply_args(conf, args)
    return conf


def test_fleet_env_args(monkeypatch):
    from dstack_amd.core.models.fleets import FleetConfiguration

    conf = FleetConfiguration.model_validate({"type": "fleet", "ssh_config": {"hosts": ["1.2.3.4"]},
                                              "env": {"A": "0", "FROM_CONF": "1"}})
    monkeypatch.setenv("FROM_ENV", "2")
    out = _fleet_args(conf, ["-e", "A=1", "--env", "FROM_ENV"])
    assert dict(out.env) == {"A": "1", "FROM_CONF": "1", "FROM_ENV": "2"}
    monkeypatch.delenv("FROM_ENV")
    with pytest.raises(ConfigurationError, match="FROM_ENV is not set"):
        _fleet_args(conf, ["--env", "FROM_ENV"])


# ---- dstack config ------------------------------------------------------------------------------
def test_dstack_config_writes_project():
    from unittest import mock

    from dstack_amd.cli import commands
    from dstack_amd.core.services.configs import ConfigManager

    parser = argparse.ArgumentParser()
    commands.register_config(parser.add_subparsers())
    args = parser.parse_args(["config", "--url", "http://127.0.0.1:31313", "--project", "project",
                              "--token", "token"])
    with mock.patch("dstack_amd.api.server.APIClient") as api:
        assert args.func(args) == 0
    api.assert_called_once()
    assert api.call_args.kwargs.get("base_url", api.call_args.args[0] if api.call_args.args else None) == \
        "http://127.0.0.1:31313"
    with open(ConfigManager().config_filepath) as f:
        cfg = yaml.safe_load(f)
    assert cfg["projects"] == [{"default": True, "name": "project", "token": "token",
                                "url": "http://127.0.0.1:31313"}]


def test_dev_environment_pins_local_vscode_version(tmp_path, monkeypatch):
    """``ide: vscode`` without ``version``: the local VS Code's commit (``code --version`` line 2)
    is pinned so the container's IDE server matches the desktop client; no ``code``: left unset."""
    from dstack_amd.core.models.configurations import DevEnvironmentConfiguration

    commit = "1a5daa3a0231a0fbba4f14db7ec463cf99d7768e"
    code = tmp_path / "code"
    code.write_text(f"#!/bin/sh\necho 1.97.2\necho {commit}\necho x64\n")
    code.chmod(0o755)
    dev = DevEnvironmentConfiguration.model_validate({"type": "dev-environment", "ide": "vscode"})
    monkeypatch.setenv("PATH", f"{tmp_path}:/usr/bin:/bin")
    assert _run_args(dev, []).version == commit
    monkeypatch.setenv("PATH", "/nonexistent")
    assert _run_args(dev, []).version is None
