"""RunSpec -> JobSpec[] (reference: ``S/services/jobs/configurators/{base,task,dev,service}.py``).

* commands: ``/bin/bash -c "<setup && commands>"`` (or the configured entrypoint);
* default image: a ROCm PyTorch image when AMD GPUs are requested (MI355X-first), else a base
  Ubuntu/Python image; images are irrelevant for the ``process`` shim driver;
* max_duration defaults: task/service off, dev-environment 6 h; stop_duration 300 s;
* tasks expand into ``nodes`` jobs per replica; services into one job per replica;
* ``${{ dstack.node_rank }}`` is interpolated into volume names/paths per job;
* the MI355X health probe is requested for jobs that take AMD GPUs on a fresh instance.
"""

from __future__ import annotations

import shlex
from typing import Dict, List, Optional

from dstack_amd.core.errors import ServerClientError
from dstack_amd.core.models.configurations import (
    DevEnvironmentConfiguration,
    PortMapping,
    ServiceConfiguration,
    TaskConfiguration,
)
from dstack_amd.core.models.images import DEFAULT_ROCM_IMAGE, check_requested_gpus
from dstack_amd.core.models.profiles import DEFAULT_STOP_DURATION, ProfileRetry, RetryEvent, SpotPolicy
from dstack_amd.core.models.resources import AcceleratorVendor
from dstack_amd.core.models.runs import AppSpec, JobSpec, Requirements, Retry, RunSpec, get_policy_map
from dstack_amd.core.models.unix import UnixUser
from dstack_amd.core.models.volumes import InstanceMountPoint, VolumeMountPoint
from dstack_amd.utils.interpolator import InterpolatorError, VariablesInterpolator

DEFAULT_MAX_DURATION_DEV = 6 * 3600
DEFAULT_AMD_IMAGE = DEFAULT_ROCM_IMAGE  # ROCm >= 7.0: gfx950 (MI350X/MI355X) support
DEFAULT_CPU_IMAGE = "python:{python}-slim"


def get_default_python_version() -> str:
    return "3.10"


def get_default_image(conf) -> str:
    gpu = conf.resources.gpu
    wants_gpu = gpu is not None and gpu.count.max != 0
    if wants_gpu and gpu.vendor in (None, AcceleratorVendor.AMD):
        return DEFAULT_AMD_IMAGE
    py = conf.python.value if conf.python else get_default_python_version()
    return DEFAULT_CPU_IMAGE.format(python=py)


def _retry(run_spec: RunSpec) -> Optional[Retry]:
    return retry_from_profile(run_spec.merged_profile)


def retry_from_profile(prof) -> Optional[Retry]:
    """``retry`` (or the deprecated ``retry_policy``) of a profile as (events, duration seconds)."""
    r = prof.retry
    if r is None and prof.retry_policy is not None and prof.retry_policy.retry:
        return Retry(on_events=[RetryEvent.NO_CAPACITY, RetryEvent.INTERRUPTION, RetryEvent.ERROR],
                     duration=int(prof.retry_policy.duration or 3600))
    if r is None or r is False:
        return None
    if r is True:
        return Retry(on_events=[RetryEvent.NO_CAPACITY, RetryEvent.INTERRUPTION, RetryEvent.ERROR], duration=3600)
    assert isinstance(r, ProfileRetry)
    return Retry(on_events=r.on_events, duration=int(r.duration or 3600))


def _duration(v, default: Optional[int]) -> Optional[int]:
    if v == "off":
        return None
    if v is None:
        return default
    return int(v)


def _shell_commands(conf, run_name: Optional[str] = None) -> List[str]:
    if isinstance(conf, DevEnvironmentConfiguration):
        from dstack_amd.server.services.jobs.ide import dev_environment_commands

        return dev_environment_commands(conf, run_name or "dev")
    return list(conf.setup) + list(conf.commands)


def _build_commands(conf, image_entrypoint: Optional[List[str]] = None, run_name: Optional[str] = None) -> List[str]:
    shell = _shell_commands(conf, run_name)
    if conf.entrypoint is not None:
        return shlex.split(conf.entrypoint) + shell
    if shell:
        return ["/bin/bash", "-c", " && ".join(shell)]
    return list(image_entrypoint or [])


def _app_specs(conf) -> List[AppSpec]:
    specs = []
    ports: List[PortMapping] = getattr(conf, "ports", []) or []
    for i, p in enumerate(ports):
        specs.append(AppSpec(port=p.container_port, map_to_port=p.local_port, app_name=f"app{i}"))
    return specs


def interpolate_job_volumes(volumes, job_num: int):
    """Per-job mount points: ``${{ dstack.job_num }}`` / ``${{ dstack.node_rank }}`` resolved in volume
    names and paths; volume names always come out as a list of alternatives (reference:
    ``S/services/jobs/configurators/base.py`` ``interpolate_job_volumes``). A bad pattern is the
    user's error (``ServerClientError``)."""
    it = VariablesInterpolator({"dstack": {"job_num": str(job_num), "node_rank": str(job_num)}})
    out = []
    for v in volumes:
        try:
            if isinstance(v, VolumeMountPoint):
                names = v.name if isinstance(v.name, list) else [v.name]
                out.append(VolumeMountPoint(name=[it.interpolate(n) for n in names], path=it.interpolate(v.path)))
            elif isinstance(v, InstanceMountPoint):
                out.append(InstanceMountPoint(instance_path=it.interpolate(v.instance_path),
                                              path=it.interpolate(v.path), optional=v.optional))
        except InterpolatorError as e:
            raise ServerClientError(f"Failed to interpolate volume {v}: {e}") from e
    return out


def get_job_specs_from_run_spec(run_spec: RunSpec, replica_num: int = 0,
                                secrets: Optional[Dict[str, str]] = None) -> List[JobSpec]:
    conf = run_spec.configuration
    prof = run_spec.merged_profile
    nodes = conf.nodes if isinstance(conf, TaskConfiguration) else 1
    spot = get_policy_map(prof.spot_policy, SpotPolicy.ONDEMAND if not isinstance(conf, TaskConfiguration)
                          else SpotPolicy.ONDEMAND)
    requirements = Requirements(resources=conf.resources, max_price=prof.max_price, spot=spot,
                                reservation=prof.reservation)
    if isinstance(conf, DevEnvironmentConfiguration):
        max_duration = _duration(prof.max_duration, DEFAULT_MAX_DURATION_DEV)
    else:
        max_duration = _duration(prof.max_duration, None)
    stop_duration = _duration(prof.stop_duration, DEFAULT_STOP_DURATION)
    env: Dict[str, str] = {}
    ns = {"secrets": dict(secrets or {}), "env": {}}
    it = VariablesInterpolator(ns, skip=["run"])
    for k, v in conf.env.items():
        if hasattr(v, "key"):  # unresolved sentinel: the client did not provide it
            continue
        env[k] = it.interpolate(str(v), return_missing=True)[0]
    image = conf.image or get_default_image(conf)
    # an image whose tag names a ROCm older than every requested GPU supports (ROCm 6.x for an
    # MI355X-only run) can never run: rejected at submission with the image to use instead
    gpu = conf.resources.gpu
    bad = check_requested_gpus(image, gpu.name if gpu is not None and (gpu.count.max or 0) > 0 else None)
    if bad:
        raise ServerClientError(bad)
    user = UnixUser.parse(conf.user) if conf.user else None
    image_entrypoint = None
    if conf.image and (not _shell_commands(conf) or user is None) and conf.entrypoint is None:
        # a custom image without commands runs its own ENTRYPOINT + CMD; its USER is the default user
        cfg = _image_config(conf)
        if cfg is not None:
            if not _shell_commands(conf):
                image_entrypoint = (cfg.entrypoint or []) + (cfg.cmd or [])
            if user is None and cfg.user:
                try:
                    user = UnixUser.parse(cfg.user)
                except ValueError:
                    user = None
    gpu_wanted = conf.resources.gpu is not None and (conf.resources.gpu.count.max or 0) > 0
    specs = []
    for job_num in range(nodes):
        job_name = f"{run_spec.run_name}-{job_num}-{replica_num}"
        specs.append(JobSpec(
            replica_num=replica_num, job_num=job_num, job_name=job_name, jobs_per_replica=nodes,
            app_specs=_app_specs(conf), user=user, commands=_build_commands(conf, image_entrypoint, run_spec.run_name),
            env=env,
            home_dir=conf.home_dir, image_name=image, privileged=conf.privileged,
            single_branch=conf.single_branch if conf.single_branch is not None
            else not isinstance(conf, DevEnvironmentConfiguration),
            max_duration=max_duration, stop_duration=stop_duration, registry_auth=conf.registry_auth,
            requirements=requirements, retry=_retry(run_spec),
            volumes=[v.model_dump(mode="json") for v in interpolate_job_volumes(conf.volumes, job_num)],
            working_dir=conf.working_dir or run_spec.working_dir,
            gpu_probe=gpu_wanted and env.get("DSTACK_GPU_PROBE", "0") == "1",
        ))
    return specs


def _image_config(conf):
    """Registry lookup (cached 80 s).  A registry that answers "no" (unknown image or tag, no
    access) fails the submission as in the reference (``jobs/configurators/base.py:_get_image_config``);
    an unreachable registry (an air-gapped server with a local image mirror on the hosts) only skips
    the lookup, and the image's own entrypoint/user are then not known to the server."""
    from dstack_amd.core.errors import DockerRegistryError, ServerClientError
    from dstack_amd.server.services.docker import get_image_config

    ra = conf.registry_auth
    try:
        return get_image_config(conf.image, ra.username if ra else None, ra.password if ra else None)
    except DockerRegistryError as e:
        raise ServerClientError(f"Error pulling configuration for image {conf.image!r} from the docker registry: {e}")
    except Exception:  # noqa: BLE001 - registry unreachable: do not block submission
        return None


def service_port(conf: ServiceConfiguration) -> int:
    return conf.port.container_port
