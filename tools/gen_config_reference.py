"""Generate docs/reference/dstack.yml.md from the configuration models (every field of every
configuration type, its type, default and description), so the reference cannot drift from the
code.  Run: python tools/gen_config_reference.py"""
import os
import sys
import types
import typing

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pydantic import BaseModel  # noqa: E402
from pydantic_core import PydanticUndefined  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "docs", "reference", "dstack.yml.md")


def _type_name(t) -> str:
    origin = typing.get_origin(t)
    args = [a for a in typing.get_args(t) if a is not type(None)]
    if origin is typing.Union or origin is types.UnionType:  # sorted: typing caches Union[int, str] == Union[str, int] by first use
        return " | ".join(sorted(_type_name(a) for a in args))
    if origin is typing.Literal:
        return " | ".join(repr(a) for a in typing.get_args(t))
    if origin in (list, typing.List):
        return f"list[{_type_name(args[0])}]" if args else "list"
    if origin in (dict, typing.Dict):
        return "dict"
    if origin is typing.Annotated:
        return _type_name(typing.get_args(t)[0])
    return getattr(t, "__name__", str(t)).replace("typing.", "")


def _default(f) -> str:
    if f.default is not PydanticUndefined and f.default is not None:
        d = f.default
        if isinstance(d, BaseModel):
            return "see below"
        if hasattr(d, "value"):
            d = d.value
        return f"`{d}`"
    if f.default_factory is not None:
        return "`[]`" if f.default_factory is list else "—"
    return "**required**" if f.is_required() else "—"


# descriptions for fields whose model carries none (kept here so the models stay lean)
DESCRIPTIONS = {
    "type": "Configuration type",
    "name": "Resource name; random for runs if omitted",
    "user": "User inside the container (`name`, `uid`, `name:group`, `uid:gid`); default: the image's USER",
    "privileged": "Run the container privileged (needed e.g. for Docker-in-Docker)",
    "entrypoint": "Override the image ENTRYPOINT; `commands` then become its arguments",
    "working_dir": "Working directory inside the container, relative to the repo root",
    "home_dir": "Home directory of the container user",
    "registry_auth": "`username` / `password` of a private registry; `${{ secrets.X }}` / `${{ env.X }}` interpolated",
    "python": "Python version of the default image (`3.9` .. `3.12`)",
    "nvcc": "Accepted for compatibility; the default image is ROCm (hipcc is always present)",
    "single_branch": "Clone only the run's branch of a remote repo",
    "env": "Environment variables: a mapping or `KEY=VALUE` / `KEY` (taken from the CLI environment) list",
    "setup": "Commands run before `commands` (deprecated: put them in `commands`)",
    "resources": "Resource requirements (section `resources` below)",
    "volumes": "Network volumes (`name` + `path`, or `name:/path`) or instance paths (`/host:/container`)",
    "ports": "Ports to forward on `dstack attach` (`8080` or `local:container`)",
    "commands": "Shell commands to run",
    "nodes": "Number of nodes of a distributed task; each gets DSTACK_NODE_RANK / DSTACK_MASTER_NODE_IP",
    "port": "The container port the service listens on (`8000` or `80:8000`)",
    "https": "Serve over HTTPS on the gateway (ACME certificate)",
    "auth": "Require a dstack user token for requests to the service",
    "replicas": "Replica count or range (`1..4`) for autoscaling",
    "scaling": "Autoscaling policy (section `scaling` below)",
    "strip_prefix": "Strip `/proxy/services/<project>/<run>` before forwarding (in-server proxy)",
    "ide": "IDE to set up: `vscode` (VS Code server at `version`, link printed on attach)",
    "init": "Commands run before the IDE is ready",
    "backends": "Backends to consider, e.g. `[remote, aws]`",
    "regions": "Regions to consider",
    "instance_types": "Instance types to consider",
    "reservation": "Capacity reservation / block id (AWS)",
    "spot_policy": "`spot`, `on-demand` or `auto` (spot first)",
    "retry_policy": "Legacy retry form (`retry` supersedes it)",
    "max_price": "Maximum price per instance-hour",
    "creation_policy": "`reuse` (only existing instances) or `reuse-or-create`",
    "termination_policy": "`destroy-after-idle` or `dont-destroy` (legacy pool settings)",
    "pool_name": "Pool to use (legacy; fleets replace pools)",
    "instance_name": "Reuse this instance of the pool (legacy)",
    "placement": "`cluster`: all instances in one network segment (placement group) for multi-node jobs",
    "ssh_config": "Hosts of an SSH fleet (on-prem MI355X nodes; section below)",
    "ssh_key": "Private key (or its path in `identity_file`) used to reach the hosts",
    "identity_file": "Path to the SSH private key",
    "hostname": "Host name or IP",
    "internal_ip": "Address other hosts of the fleet reach this one at (multi-node)",
    "network": "Subnet (`10.0.0.0/24`) of the fleet's internal interface, for multi-node jobs",
    "backend": "Backend that provisions the resource",
    "region": "Region of the resource",
    "size": "Volume size (`100GB`)",
    "domain": "Wildcard domain of the gateway (`*.example.com` points at it)",
    "default": "Make this the project's default gateway",
    "public_ip": "Give the gateway a public IP (`false`: private gateway, AWS)",
    "certificate": "`lets-encrypt` (default) or `acm` with an ARN",
    "cpu": "CPU cores (`4`, `2..`)",
    "memory": "RAM (`64GB..`)",
    "shm_size": "Size of /dev/shm (e.g. `16GB` for NCCL/RCCL and dataloaders)",
    "gpu": "GPU requirement (`MI355X:8`, `amd:192GB..:1..`; section `resources.gpu`)",
    "disk": "Disk requirement (`200GB..`)",
    "count": "Number of GPUs (`8`, `1..`)",
    "total_memory": "Total GPU memory over all GPUs (`1TB..`)",
    "compute_capability": "NVIDIA compute capability (not used for AMD GPUs)",
    "target": "Target value of the metric per replica (requests per second)",
    "scale_up_delay": "Seconds the metric must stay above target before adding a replica",
    "scale_down_delay": "Seconds the metric must stay below target before removing a replica",
    "on_events": "Retry on `no-capacity`, `interruption`, `error`",
}


def section(title: str, model, skip=(), extra=None) -> str:
    rows = [f"## {title}\n", "| Field | Type | Default | Description |", "|---|---|---|---|"]
    for name, f in model.model_fields.items():
        if name in skip or name.startswith("_"):
            continue
        key = f.alias or name
        desc = (f.description or (extra or {}).get(name) or DESCRIPTIONS.get(name, "")).replace("|", "\\|").replace("\n", " ")
        rows.append(f"| `{key}` | `{_type_name(f.annotation)}` | {_default(f)} | {desc} |")
    return "\n".join(rows) + "\n"


def render() -> str:
    from dstack_amd.core.models.configurations import (
        DevEnvironmentConfiguration,
        ServiceConfiguration,
        TaskConfiguration,
    )
    from dstack_amd.core.models.fleets import FleetConfiguration, SSHHostParams, SSHParams
    from dstack_amd.core.models.gateways import GatewayConfiguration
    from dstack_amd.core.models.profiles import Profile, ProfileRetry
    from dstack_amd.core.models.resources import DiskSpec, GPUSpec, ResourcesSpec
    from dstack_amd.core.models.services import ScalingSpec
    from dstack_amd.core.models.volumes import VolumeConfiguration

    parts = ["# `.dstack.yml` reference\n",
             "Generated from the configuration models by `tools/gen_config_reference.py`; every field "
             "the server accepts is listed.  Run configurations (`task`, `service`, `dev-environment`) "
             "also accept every profile field (last section) at the top level.\n"]
    parts.append(section("type: task", TaskConfiguration))
    parts.append(section("type: service", ServiceConfiguration))
    parts.append(section("type: dev-environment", DevEnvironmentConfiguration))
    parts.append(section("type: fleet", FleetConfiguration))
    ssh = {"port": "SSH port (22)", "user": "SSH user on the hosts", "hosts": "Host names / IPs, or mappings (next section)"}
    parts.append(section("fleet `ssh_config`", SSHParams, extra=ssh))
    parts.append(section("fleet `ssh_config.hosts[]` (mapping form)", SSHHostParams, extra=ssh))
    parts.append(section("type: volume", VolumeConfiguration))
    parts.append(section("type: gateway", GatewayConfiguration))
    parts.append(section("`resources`", ResourcesSpec))
    parts.append(section("`resources.gpu` (mapping form; the string form is `[vendor:]name[:memory][:count]`)",
                         GPUSpec))
    parts.append(section("`resources.disk`", DiskSpec))
    parts.append(section("service `scaling`", ScalingSpec))
    parts.append(section("`retry`", ProfileRetry))
    parts.append(section("Profile fields (`.dstack/profiles.yml` entries and run-configuration top level)", Profile))
    return "\n".join(parts)


def main():
    with open(OUT, "w") as f:
        f.write(render())
    print(OUT)


if __name__ == "__main__":
    main()
