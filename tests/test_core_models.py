"""Configuration grammar tests (reference: ``src/tests/_internal/core/models/test_{resources,
configurations,unix}.py``, ``utils/test_interpolator.py``) plus every example ``.dstack.yml`` shipped
in the reference repo (read as YAML text with ``yaml.safe_load``)."""

import os

import pytest
import yaml
from pydantic import TypeAdapter, ValidationError

from dstack_amd.core.errors import ConfigurationError
from dstack_amd.core.models.configurations import (
    DevEnvironmentConfiguration,
    ServiceConfiguration,
    TaskConfiguration,
    parse_apply_configuration,
    parse_run_configuration,
)
from dstack_amd.core.models.envs import Env
from dstack_amd.core.models.resources import (
    AcceleratorVendor,
    ComputeCapability,
    GPUSpec,
    Memory,
    Range,
    ResourcesSpec,
)
from dstack_amd.core.models.unix import UnixUser
from dstack_amd.utils.interpolator import InterpolatorError, VariablesInterpolator


def parse(tp, v):
    return TypeAdapter(tp).validate_python(v)


# ---- Memory / ComputeCapability / Range ------------------------------------------------------
@pytest.mark.parametrize("v,expected", [("512MB", 0.5), ("16 Gb", 16.0), ("1 TB ", 1024.0), (1.5, 1.5), (1, 1.0),
                                        ("288GB", 288.0)])
def test_memory(v, expected):
    assert parse(Memory, v) == expected


def test_memory_invalid():
    with pytest.raises(ValidationError):
        parse(Memory, "1.5xb")


@pytest.mark.parametrize("v,expected", [("3.5", (3, 5)), (8.0, (8, 0)), ((7, 5), (7, 5))])
def test_compute_capability(v, expected):
    assert parse(ComputeCapability, v) == expected


@pytest.mark.parametrize("v", ["3.5.1", "3.x"])
def test_compute_capability_invalid(v):
    with pytest.raises(ValidationError):
        parse(ComputeCapability, v)


@pytest.mark.parametrize("v,expected", [(1, (1, 1)), ("1", (1, 1)), ("1..", (1, None)), ("..1", (None, 1)),
                                        ({"min": 1, "max": 3}, (1, 3))])
def test_int_range(v, expected):
    r = parse(Range[int], v)
    assert (r.min, r.max) == expected
    assert isinstance(str(r), str)


@pytest.mark.parametrize("v", ["..", "1...3", "3..1"])
def test_int_range_invalid(v):
    with pytest.raises(ValidationError):
        parse(Range[int], v)


@pytest.mark.parametrize("v,expected", [("512MB", (0.5, 0.5)), ("512MB..", (0.5, None)), ("..1 TB", (None, 1024.0)),
                                        ("512..1 TB", (512.0, 1024.0)), ({"min": "512MB", "max": "1TB"}, (0.5, 1024.0))])
def test_memory_range(v, expected):
    r = parse(Range[Memory], v)
    assert (r.min, r.max) == expected


# ---- GPU spec grammar -------------------------------------------------------------------------
def test_gpu_count_only():
    assert parse(GPUSpec, "1") == parse(GPUSpec, {"count": 1})


@pytest.mark.parametrize("v,vendor", [("amd", AcceleratorVendor.AMD), ("AMD:2", AcceleratorVendor.AMD),
                                      ("nvidia", AcceleratorVendor.NVIDIA), ("tpu", AcceleratorVendor.GOOGLE)])
def test_gpu_vendor_string(v, vendor):
    assert parse(GPUSpec, v).vendor == vendor


def test_gpu_mi355x_infers_amd():
    g = parse(GPUSpec, "MI355X:8")
    assert g.vendor == AcceleratorVendor.AMD
    assert g.name == ["MI355X"]
    assert (g.count.min, g.count.max) == (8, 8)


def test_gpu_full_string():
    g = parse(GPUSpec, "amd:MI300X,MI355X:192GB..:2..8")
    assert g.vendor == AcceleratorVendor.AMD
    assert set(g.name) == {"MI300X", "MI355X"}
    assert g.memory.min == 192.0
    assert (g.count.min, g.count.max) == (2, 8)


def test_gpu_object_form():
    g = parse(GPUSpec, {"name": "MI355X", "count": "1..2", "memory": "288GB"})
    assert g.vendor == AcceleratorVendor.AMD and g.count.max == 2


def test_resources_defaults_and_shm():
    r = parse(ResourcesSpec, {"gpu": "MI355X:8", "shm_size": "16GB", "disk": "500GB.."})
    assert r.shm_size == 16.0
    assert r.disk.size.min == 500.0
    assert r.cpu.min >= 1
    assert "MI355X" in r.pretty_format()


# ---- configurations ---------------------------------------------------------------------------
def test_task_commands_and_env():
    c = parse_run_configuration({"type": "task", "commands": ["python train.py"], "env": ["A=1", "HF_TOKEN"],
                                 "resources": {"gpu": "MI355X:8"}, "nodes": 2})
    assert isinstance(c, TaskConfiguration)
    assert c.nodes == 2
    assert c.env["A"] == "1"


def test_service_replicas_and_scaling():
    def conf(replicas, scaling=None):
        d = {"type": "service", "commands": ["python -m http.server"], "port": 8000, "replicas": replicas}
        if scaling:
            d["scaling"] = scaling
        return d

    r = parse_run_configuration(conf(1)).replicas
    assert (r.min, r.max) == (1, 1)
    r = parse_run_configuration(conf("2")).replicas
    assert (r.min, r.max) == (2, 2)
    c = parse_run_configuration(conf("0..4", {"metric": "rps", "target": 10}))
    assert isinstance(c, ServiceConfiguration)
    assert (c.replicas.min, c.replicas.max) == (0, 4)
    with pytest.raises((ConfigurationError, ValidationError, ValueError)):
        parse_run_configuration(conf("1..3"))  # a replica range requires scaling


def test_service_gpu_util_scaling():
    c = parse_run_configuration({"type": "service", "commands": ["x"], "port": 80, "replicas": "1..8",
                                 "scaling": {"metric": "gpu_util", "target": 70}})
    assert c.scaling.metric == "gpu_util"


def test_dev_environment():
    c = parse_run_configuration({"type": "dev-environment", "ide": "vscode"})
    assert isinstance(c, DevEnvironmentConfiguration)


def test_unknown_field_rejected():
    with pytest.raises((ConfigurationError, ValidationError)):
        parse_run_configuration({"type": "task", "commands": ["x"], "commnds": ["y"]})


def _reference_examples():
    out = []
    for root, _, files in os.walk("/root/reference"):
        for fn in files:
            if fn.endswith(".dstack.yml"):
                out.append(os.path.join(root, fn))
    return sorted(out)


# a reference example with a typo (`command:` instead of `commands:`) that the reference's own
# strict models reject as well
_KNOWN_INVALID = {"examples/deployment/vllm/amd/build-vllm.dstack.yml"}


@pytest.mark.skipif(not os.path.isdir("/root/reference"), reason="reference checkout not mounted")
@pytest.mark.parametrize("path", _reference_examples())
def test_reference_example_configurations(path):
    with open(path) as f:
        data = yaml.safe_load(f)
    rel = os.path.relpath(path, "/root/reference")
    if rel in _KNOWN_INVALID:
        with pytest.raises((ConfigurationError, ValidationError)):
            parse_apply_configuration(data)
        return
    conf = parse_apply_configuration(data)
    assert conf.type == data["type"]


# ---- env / unix user / interpolation ----------------------------------------------------------
def test_env_forms():
    assert Env(["A=1", "B=x=y"])["B"] == "x=y"
    assert Env({"A": 1})["A"] == "1"


@pytest.mark.parametrize("v,user,uid,gid", [("root", "root", None, None), ("1000", None, 1000, None),
                                            ("1000:1000", None, 1000, 1000), ("user:group", "user", None, None)])
def test_unix_user(v, user, uid, gid):
    u = UnixUser.parse(v)
    assert u.username == user and u.uid == uid and u.gid == gid


@pytest.mark.parametrize("v", ["a:b:c", ":group", "-1"])
def test_unix_user_invalid(v):
    with pytest.raises(ValueError):
        UnixUser.parse(v)


def _interp():
    return VariablesInterpolator({"run": {"args": "qwerty"}, "secrets": {"tok": "abc"}}, skip=["env"])


def test_interpolator_plain_and_bash():
    assert _interp().interpolate("") == ""
    s = "echo $FOO ${BAR} $((1+2))"
    assert _interp().interpolate(s) == s


def test_interpolator_escape_and_values():
    assert _interp().interpolate("$${{ENV}}") == "${{ENV}}"
    assert _interp().interpolate("${{ run.args }}") == "qwerty"
    assert _interp().interpolate("${{ secrets.tok }}") == "abc"
    assert _interp().interpolate("${{ env.name }}") == "${{ env.name }}"  # skipped namespace stays


def test_interpolator_missing_and_errors():
    s, missing = VariablesInterpolator({"run": {}}).interpolate("${{ run.nope }}", return_missing=True)
    assert s == "" and missing == ["run.nope"]
    with pytest.raises(InterpolatorError):
        _interp().interpolate("${{ run.args ")
    with pytest.raises(InterpolatorError):
        _interp().interpolate("${{ run.ar-gs }}")


def _own_examples():
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples")
    return sorted(os.path.join(d, f) for d, _, fs in os.walk(root) for f in fs if f.endswith(".dstack.yml"))


@pytest.mark.parametrize("path", _own_examples())
def test_own_example_configurations(path):
    with open(path) as f:
        data = yaml.safe_load(f)
    conf = parse_apply_configuration(data)
    assert conf.type == data["type"]


def test_configuration_reference_doc_is_current():
    """docs/reference/dstack.yml.md is generated from the models: regenerate it
    (``python tools/gen_config_reference.py``) after changing a configuration field."""
    import importlib.util

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("gen_config_reference",
                                                  os.path.join(root, "tools", "gen_config_reference.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    with open(os.path.join(root, "docs", "reference", "dstack.yml.md")) as f:
        assert f.read() == mod.render()
