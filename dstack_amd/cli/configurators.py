"""``dstack apply`` configurators (reference: ``cli/services/configurators/{run,fleet,gateway,volume}.py``,
``cli/services/profile.py``, ``cli/services/repos.py``).

Each configurator registers its CLI overrides, shows a plan, asks for confirmation and applies.
The run configurator then follows the run: waits for RUNNING, forwards ports (attach) and streams
logs until the run finishes; Ctrl-C offers to stop the run.  The process exit code is the job's.
"""

from __future__ import annotations

import argparse
import os
import signal
import sys
import time
from pathlib import Path
from typing import Dict, List, Optional

import yaml

from dstack_amd.api import Client
from dstack_amd.cli.utils import confirm_ask, console, fleets_table, plan_table, print_table, status_text
from dstack_amd.core.errors import CLIError, ConfigurationError
from dstack_amd.core.models.configurations import PortMapping
from dstack_amd.core.models.envs import Env
from dstack_amd.core.models.profiles import CreationPolicy, Profile, ProfilesConfig, SpotPolicy, TerminationPolicy
from dstack_amd.core.models.repos import LocalRepo, RemoteRepo, Repo, RepoError, VirtualRepo
from dstack_amd.core.models.runs import JobStatus, RunStatus


# ---- profile arguments (cli/services/profile.py) ----------------------------------------------
def register_profile_args(parser: argparse.ArgumentParser):
    g = parser.add_argument_group("Profile")
    g.add_argument("--profile", metavar="NAME", default=os.getenv("DSTACK_PROFILE"),
                   help="Profile from .dstack/profiles.yml (default: $DSTACK_PROFILE)")
    g.add_argument("--max-price", type=float, metavar="PRICE", help="Max price per hour, $")
    g.add_argument("--max-duration", metavar="DURATION", help="Max run duration, e.g. 72h or off")
    g.add_argument("-b", "--backend", action="append", dest="backends", metavar="NAME")
    g.add_argument("-r", "--region", action="append", dest="regions", metavar="NAME")
    g.add_argument("--instance-type", action="append", dest="instance_types", metavar="NAME")
    pools = parser.add_argument_group("Pools").add_mutually_exclusive_group()
    pools.add_argument("--pool", dest="pool_name", metavar="POOL")
    pools.add_argument("-R", "--reuse", dest="creation_policy_reuse", action="store_true",
                       help="Only reuse existing (idle) instances")
    pools.add_argument("--dont-destroy", dest="dont_destroy", action="store_true")
    pools.add_argument("--idle-duration", dest="idle_duration", metavar="DURATION")
    pools.add_argument("--instance", dest="instance_name", metavar="NAME")
    spot = parser.add_argument_group("Spot policy").add_mutually_exclusive_group()
    spot.add_argument("--spot", action="store_const", dest="spot_policy", const=SpotPolicy.SPOT)
    spot.add_argument("--on-demand", action="store_const", dest="spot_policy", const=SpotPolicy.ONDEMAND)
    spot.add_argument("--spot-auto", action="store_const", dest="spot_policy", const=SpotPolicy.AUTO)
    spot.add_argument("--spot-policy", dest="spot_policy", type=SpotPolicy)
    retry = parser.add_argument_group("Retry policy").add_mutually_exclusive_group()
    retry.add_argument("--retry", action="store_const", dest="retry_policy", const=True)
    retry.add_argument("--no-retry", action="store_const", dest="retry_policy", const=False)
    retry.add_argument("--retry-duration", dest="retry_duration", metavar="DURATION")


def load_profile(repo_dir: str, name: Optional[str]) -> Profile:
    """Repo profile, then the user's global one, then an empty default (``api.utils.load_profile``)."""
    from dstack_amd.api.utils import load_profile as _load

    try:
        return _load(repo_dir, name)
    except ConfigurationError as e:
        raise CLIError(str(e)) from e


def apply_profile_args(args, profile: Profile):
    """CLI profile flags onto ``profile``; the changed fields are re-validated through the model
    (``1h`` → seconds, backend names → enum, retry mapping → ``ProfileRetry``)."""
    upd = {}
    if args.max_price is not None:
        upd["max_price"] = args.max_price
    if args.max_duration is not None:
        upd["max_duration"] = args.max_duration
    if args.backends:
        upd["backends"] = args.backends
    if args.regions:
        upd["regions"] = args.regions
    if args.instance_types:
        upd["instance_types"] = args.instance_types
    if args.pool_name:
        upd["pool_name"] = args.pool_name
    if args.creation_policy_reuse:
        upd["creation_policy"] = CreationPolicy.REUSE
    if args.dont_destroy:
        upd["termination_policy"] = TerminationPolicy.DONT_DESTROY
    if args.idle_duration is not None:
        upd["idle_duration"] = args.idle_duration
    if args.instance_name:
        upd["instance_name"] = args.instance_name
        upd["creation_policy"] = CreationPolicy.REUSE
    if args.spot_policy is not None:
        upd["spot_policy"] = args.spot_policy
    events = ["no-capacity", "interruption", "error"]
    if args.retry_policy is not None:
        upd["retry"] = {"on_events": events, "duration": args.retry_duration} if args.retry_policy else False
    elif args.retry_duration:
        upd["retry"] = {"on_events": events, "duration": args.retry_duration}
    if upd:
        merged = type(profile).model_validate({**profile.model_dump(), **upd})
        for k in upd:
            setattr(profile, k, getattr(merged, k))


# ---- repo selection (cli/services/repos.py) ---------------------------------------------------
def register_repo_args(parser: argparse.ArgumentParser):
    g = parser.add_argument_group("Repo Options")
    g.add_argument("-P", "--repo", help="Repo path (default: the current directory)")
    g.add_argument("--repo-branch", dest="repo_branch")
    g.add_argument("--repo-hash", dest="repo_hash")
    g.add_argument("--no-repo", dest="no_repo", action="store_true", help="Run without a repo (no code upload)")


def get_repo(args, configuration_dir: str) -> Repo:
    if getattr(args, "no_repo", False):
        return VirtualRepo()
    path = os.path.abspath(args.repo or os.getcwd())
    from dstack_amd.core.services.configs import ConfigManager

    rc = ConfigManager().get_repo_config(path)
    if rc is not None and rc.repo_type == "local":
        return LocalRepo(path, rc.repo_id)
    if (Path(path) / ".git").exists():
        try:
            repo = RemoteRepo(path, repo_id=rc.repo_id if rc else None)
            if args.repo_branch:
                repo.run_repo_data.repo_branch = args.repo_branch
            if args.repo_hash:
                repo.run_repo_data.repo_hash = args.repo_hash
            return repo
        except RepoError:
            pass  # no origin: upload the working tree instead
    return LocalRepo(path)


# ---- configuration loading --------------------------------------------------------------------
def load_configuration(path: str):
    from dstack_amd.core.models.configurations import parse_apply_configuration

    p = Path(path)
    if not p.exists():
        raise ConfigurationError(f"Configuration file {path} does not exist")
    try:
        data = yaml.safe_load(p.read_text())
    except yaml.YAMLError as e:
        raise ConfigurationError(f"Invalid YAML in {path}: {e}") from e
    if not isinstance(data, dict):
        raise ConfigurationError(f"{path} must contain a YAML mapping")
    return parse_apply_configuration(data)


def find_default_configuration(cwd: str) -> Optional[str]:
    for name in (".dstack.yml", ".dstack.yaml"):
        if os.path.exists(os.path.join(cwd, name)):
            return os.path.join(cwd, name)
    return None


# ---- run configuration overrides --------------------------------------------------------------
def apply_env_args(conf, env_args: List[str]) -> None:
    """``-e KEY=VALUE`` sets, ``-e KEY`` copies the local value (error if unset); ``env: [KEY]``
    entries of the configuration without a value are filled from the local environment too."""
    if env_args:
        env = Env(conf.env)
        for e in env_args:
            if "=" in e:
                k, v = e.split("=", 1)
                env[k] = v
            elif e in os.environ:
                env[e] = os.environ[e]
            else:
                raise ConfigurationError(f"{e} is not set in the local environment")
        conf.env = env
    try:
        conf.env = Env(conf.env).resolve(os.environ)
    except (KeyError, ValueError) as e:
        raise ConfigurationError(f"Environment variable not set locally: {e}") from e


def merge_ports(conf_ports, arg_ports: List[PortMapping]) -> List[PortMapping]:
    """``-p`` mappings replace the configuration's mapping of the same container port; two ``-p``
    for one container port, or one local port used twice, is an error."""
    by_container: Dict[int, PortMapping] = {}
    for p in arg_ports:
        if p.container_port in by_container:
            raise ConfigurationError(f"Container port {p.container_port} is mapped more than once")
        by_container[p.container_port] = p
    merged = {p.container_port: p for p in conf_ports}
    merged.update(by_container)
    local = [p.local_port for p in merged.values() if p.local_port is not None]
    dup = {x for x in local if local.count(x) > 1}
    if dup:
        raise ConfigurationError(f"Local port(s) {sorted(dup)} are mapped more than once")
    return list(merged.values())


def interpolate_registry_auth(conf) -> None:
    """``registry_auth`` may reference the run's env: ``password: ${{ env.REGISTRY_TOKEN }}``."""
    auth = getattr(conf, "registry_auth", None)
    if auth is None:
        return
    from dstack_amd.utils.interpolator import InterpolatorError, VariablesInterpolator

    it = VariablesInterpolator({"env": {k: str(v) for k, v in dict(Env(conf.env)).items()}}, skip=["secrets"])
    try:
        conf.registry_auth = type(auth)(username=it.interpolate_or_error(auth.username),
                                        password=it.interpolate_or_error(auth.password))
    except InterpolatorError as e:
        raise ConfigurationError(f"registry_auth: {e}") from e


def validate_gpu_vendor_and_image(conf) -> None:
    """Infer ``resources.gpu.vendor`` from the names when they agree on one vendor (done by the
    GPU spec model) and require ``image`` for a non-AMD GPU: the default image here is the ROCm
    base image, so only AMD GPUs can run without one (the reference's rule is the mirror image: a
    CUDA default image, ``image`` required for AMD)."""
    gpu = conf.resources.gpu if conf.resources is not None else None
    if gpu is None or getattr(conf, "image", None):
        return
    if gpu.count.max == 0:
        return
    vendor = gpu.vendor.value if gpu.vendor is not None else None
    if vendor is not None and vendor != "amd":
        raise ConfigurationError(f"`image` is required if `resources.gpu.vendor` is `{vendor}` "
                                 "(the default image is ROCm-only)")


def detect_vscode_version(exe: str = "code") -> Optional[str]:
    """The commit hash of the local VS Code (second line of ``code --version``), or None."""
    import subprocess

    try:
        r = subprocess.run([exe, "--version"], capture_output=True, text=True, timeout=20)
    except (OSError, subprocess.TimeoutExpired):
        return None
    lines = r.stdout.splitlines()
    if r.returncode != 0 or len(lines) < 2:
        return None
    return lines[1].strip() or None


# ---- run configurator -------------------------------------------------------------------------
class RunConfigurator:
    TYPES = ("task", "service", "dev-environment")

    @staticmethod
    def register_args(parser: argparse.ArgumentParser):
        g = parser.add_argument_group("Run Options")
        g.add_argument("-n", "--name", dest="run_name", help="Run name")
        g.add_argument("--max-offers", type=int, default=3, help="Number of offers to show in the plan")
        g.add_argument("-e", "--env", action="append", default=[], metavar="KEY[=VALUE]",
                       help="Environment variable (repeatable)")
        g.add_argument("--gpu", help="GPU requirement, e.g. MI355X:8 or amd:192GB..:1..")
        g.add_argument("--disk", help="Disk size requirement, e.g. 200GB..")
        g.add_argument("-p", "--port", action="append", default=[], dest="ports", metavar="[LOCAL:]CONTAINER")
        register_profile_args(parser)

    @staticmethod
    def apply_args(conf, args) -> None:
        """CLI overrides onto the configuration (reference: ``BaseRunConfigurator.apply_args``,
        ``cli/services/configurators/run.py``): ``-e`` adds/overrides env vars, ``-p`` replaces the
        mapping of the same container port, ``--gpu``/``--disk`` replace the requirement; then
        ``${{ env.X }}`` in ``registry_auth`` is resolved and the GPU vendor / image pair checked."""
        apply_env_args(conf, args.env)
        res = {k: v for k, v in (("gpu", args.gpu), ("disk", args.disk)) if v}
        if res:
            conf.resources = type(conf.resources).model_validate({**conf.resources.model_dump(), **res})
        if args.ports and hasattr(conf, "ports"):
            conf.ports = merge_ports(conf.ports, [PortMapping.parse(p) for p in args.ports])
        interpolate_registry_auth(conf)
        validate_gpu_vendor_and_image(conf)
        if getattr(conf, "type", None) == "dev-environment" and conf.ide == "vscode" and conf.version is None:
            # the IDE server in the container matches the local VS Code (commit hash), so the
            # desktop client attaches without reinstalling it
            conf.version = detect_vscode_version()
            if conf.version is None:
                console.print("[secondary]Unable to detect the VS Code version and pre-install extensions. "
                              "Run [code]Shell Command: Install 'code' command in PATH[/] from the VS Code "
                              "Command Palette to fix it.[/]")

    def apply(self, client: Client, conf, conf_path: str, args) -> int:
        self.apply_args(conf, args)
        repo = get_repo(args, os.path.dirname(os.path.abspath(conf_path)))
        profile = load_profile(repo.repo_dir or os.getcwd(), args.profile) or Profile(name="default")
        apply_profile_args(args, profile)
        run_name = args.run_name or conf.name
        with console.status("Getting run plan..."):
            plan = client.runs.get_plan(conf, repo, configuration_path=conf_path, profile=profile, run_name=run_name,
                                        max_offers=args.max_offers)
        print_table(plan_table(plan, args.max_offers))
        stop_first = None
        if plan.current_resource is not None and not plan.current_resource.status.is_finished():
            if plan.action and plan.action.value == "update":
                question = f"Active run [code]{plan.run_spec.run_name}[/] already exists. Update it?"
            else:  # not updatable in place: stop it, wait, then submit the new spec
                stop_first = plan.run_spec.run_name
                question = f"Active run [code]{stop_first}[/] already exists and cannot be updated in place. " \
                           "Stop and override the run?"
            if not args.yes and not confirm_ask(question):
                console.print("\nExiting...")
                return 0
        elif not args.yes and not confirm_ask("Submit the run?" if plan.job_plans[0].offers else
                                              "No offers right now. Submit anyway (waits for capacity)?"):
            console.print("\nExiting...")
            return 0
        if stop_first is not None:
            with console.status("Stopping run..."):
                old = client.runs.get(stop_first)
                if old is not None:
                    old.stop(abort=False)
                while old is not None and not old.status.is_finished():
                    time.sleep(1)
                    old = client.runs.get(stop_first)
            plan.current_resource = None
        with console.status("Submitting run..."):
            run = client.runs.exec_plan(plan, repo, force=args.force)
        name = run.name
        if args.detach:
            console.print(f"Run [code]{name}[/] submitted, detaching...")
            return 0
        return follow_run(client, run, attach=True)


def follow_run(client: Client, run, attach: bool = True) -> int:
    """Wait for the run to start, attach, stream logs; Ctrl-C asks whether to stop the run."""
    name = run.name
    interrupted = {"n": 0}

    def on_sigint(signum, frame):
        interrupted["n"] += 1
        raise KeyboardInterrupt

    prev = signal.signal(signal.SIGINT, on_sigint)
    try:
        with console.status(f"Launching [code]{name}[/]...") as st:
            while True:
                run.refresh()
                st.update(f"Launching [code]{name}[/] ({status_text(run.status.value)})")
                if run.status.is_finished() or run.status == RunStatus.RUNNING:
                    break
                sub = run.model.latest_job_submission
                if sub is not None and sub.status in (JobStatus.RUNNING,):
                    break
                time.sleep(0.25)
        if attach and run.status == RunStatus.RUNNING:
            try:
                if run.attach():
                    for cport, lport in (run.ports or {}).items():
                        console.print(f"Forwarded port {cport} -> [link]http://127.0.0.1:{lport}[/]")
                if run.service_url:
                    console.print(f"Service is published at [link]{run.service_url}[/]")
            except Exception as e:  # noqa: BLE001 - attaching is best-effort; logs still stream
                console.print(f"[warning]Could not attach: {e}[/]")
        for chunk in run.logs(follow=True, poll=0.3):
            sys.stdout.buffer.write(chunk)
            sys.stdout.flush()
        run.refresh()
    except KeyboardInterrupt:
        try:
            if confirm_ask(f"\nStop the run [code]{name}[/] before detaching?"):
                with console.status("Stopping..."):
                    run.stop(abort=False)
                    run.wait(timeout=120)
                console.print(f"Run [code]{name}[/] stopped")
            else:
                console.print(f"Detached from [code]{name}[/]")
        except KeyboardInterrupt:
            run.stop(abort=True)
            console.print(f"Run [code]{name}[/] aborted")
        return 0
    finally:
        signal.signal(signal.SIGINT, prev)
        run.detach()
    return _exit_code(run)


def _exit_code(run) -> int:
    st = run.status
    if st == RunStatus.DONE:
        return 0
    sub = run.model.latest_job_submission
    console.print(f"Run [code]{run.name}[/] {status_text(st.value, run.model.error, sub.exit_status if sub else None)}")
    if sub is not None and sub.termination_reason_message:
        console.print(f"[error]{sub.termination_reason_message}[/]")
    if sub is not None and sub.exit_status not in (None, 0):
        return int(sub.exit_status)
    return 1


# ---- fleet / gateway / volume -----------------------------------------------------------------
class FleetConfigurator:
    TYPES = ("fleet",)

    @staticmethod
    def register_args(parser):
        parser.add_argument_group("Fleet Options").add_argument(
            "-e", "--env", action="append", default=[], metavar="KEY[=VALUE]",
            help="Environment variable for the fleet's hosts (repeatable)")

    @staticmethod
    def apply_args(conf, args) -> None:
        apply_env_args(conf, getattr(args, "env", None) or [])

    def apply(self, client: Client, conf, conf_path: str, args) -> int:
        from dstack_amd.core.models.fleets import FleetSpec

        self.apply_args(conf, args)
        if conf.name is None:
            conf.name = Path(conf_path).stem.replace(".dstack", "").replace("_", "-") or "fleet"
        _resolve_ssh_keys(conf)
        spec = FleetSpec(configuration=conf, configuration_path=conf_path)
        plan = client.api.fleets.get_plan(client.project, spec)
        if plan.current_resource is not None:
            if not args.yes and not confirm_ask(f"Fleet [code]{conf.name}[/] exists. Re-create it?"):
                return 0
            client.api.fleets.delete(client.project, [conf.name])
            _wait_deleted(lambda: client.api.fleets.list(client.project), conf.name)
        elif not args.yes and not confirm_ask(f"Create the fleet [code]{conf.name}[/]?"):
            return 0
        fleet = client.api.fleets.create(client.project, spec)
        if args.detach:
            console.print(f"Fleet [code]{fleet.name}[/] is being provisioned, detaching...")
            return 0
        deadline = time.time() + 1800
        with console.status(f"Provisioning [code]{fleet.name}[/]..."):
            while time.time() < deadline:
                fleet = client.api.fleets.get(client.project, fleet.name)
                states = {i.status.value for i in fleet.instances}
                if fleet.instances and states <= {"idle", "busy", "terminated"}:
                    break
                time.sleep(1)
        print_table(fleets_table([fleet]))
        failed = [i for i in fleet.instances if i.status.value == "terminated"]
        return 1 if failed else 0

    def delete(self, client: Client, conf, args) -> int:
        if not args.yes and not confirm_ask(f"Delete the fleet [code]{conf.name}[/]?"):
            return 0
        client.api.fleets.delete(client.project, [conf.name])
        console.print(f"Fleet [code]{conf.name}[/] deleted")
        return 0


def _read_ssh_key(identity_file: str):
    """``identity_file`` -> SSHKey with the private key's contents (and the ``.pub`` next to it)."""
    from dstack_amd.core.models.fleets import SSHKey

    path = os.path.expanduser(identity_file)
    try:
        with open(path) as f:
            private = f.read()
    except OSError as e:
        raise ConfigurationError(f"Cannot read identity_file {identity_file}: {e}") from e
    public = ""
    if os.path.exists(path + ".pub"):
        with open(path + ".pub") as f:
            public = f.read().strip()
    return SSHKey(public=public, private=private)


def _resolve_ssh_keys(conf):
    """The fleet's ``identity_file``s are read HERE, on the client; the server gets key contents."""
    sc = getattr(conf, "ssh_config", None)
    if sc is None:
        return
    if sc.ssh_key is None and sc.identity_file:
        sc.ssh_key = _read_ssh_key(sc.identity_file)
    for h in sc.hosts:
        if not isinstance(h, str) and h.ssh_key is None and h.identity_file:
            h.ssh_key = _read_ssh_key(h.identity_file)


class GatewayConfigurator:
    TYPES = ("gateway",)

    @staticmethod
    def register_args(parser):
        pass

    def apply(self, client: Client, conf, conf_path: str, args) -> int:
        if conf.name is None:
            raise ConfigurationError("gateway configurations need a name")
        existing = [g for g in client.api.gateways.list(client.project) if g.name == conf.name]
        if existing:
            if not args.yes and not confirm_ask(f"Gateway [code]{conf.name}[/] exists. Re-create it?"):
                return 0
            client.api.gateways.delete(client.project, [conf.name])
        elif not args.yes and not confirm_ask(f"Create the gateway [code]{conf.name}[/]?"):
            return 0
        gw = client.api.gateways.create(client.project, conf)
        console.print(f"Gateway [code]{gw.name}[/] {gw.status.value}")
        return 0

    def delete(self, client: Client, conf, args) -> int:
        if not args.yes and not confirm_ask(f"Delete the gateway [code]{conf.name}[/]?"):
            return 0
        client.api.gateways.delete(client.project, [conf.name])
        console.print(f"Gateway [code]{conf.name}[/] deleted")
        return 0


class VolumeConfigurator:
    TYPES = ("volume",)

    @staticmethod
    def register_args(parser):
        pass

    def apply(self, client: Client, conf, conf_path: str, args) -> int:
        if conf.name is None:
            raise ConfigurationError("volume configurations need a name")
        existing = [v for v in client.api.volumes.list(client.project) if v.name == conf.name]
        if existing:
            console.print(f"Volume [code]{conf.name}[/] already exists ({existing[0].status.value})")
            return 0
        if not args.yes and not confirm_ask(f"Create the volume [code]{conf.name}[/]?"):
            return 0
        vol = client.api.volumes.create(client.project, conf)
        if not args.detach:
            with console.status(f"Creating [code]{vol.name}[/]..."):
                for _ in range(600):
                    vol = client.api.volumes.get(client.project, vol.name)
                    if vol.status.value in ("active", "failed"):
                        break
                    time.sleep(1)
        console.print(f"Volume [code]{vol.name}[/] {vol.status.value} {vol.status_message or ''}")
        return 0 if vol.status.value != "failed" else 1

    def delete(self, client: Client, conf, args) -> int:
        if not args.yes and not confirm_ask(f"Delete the volume [code]{conf.name}[/]?"):
            return 0
        client.api.volumes.delete(client.project, [conf.name])
        console.print(f"Volume [code]{conf.name}[/] deleted")
        return 0


def _wait_deleted(list_fn, name: str, timeout: float = 300):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if all(x.name != name for x in list_fn()):
            return
        time.sleep(1)


CONFIGURATORS = [RunConfigurator, FleetConfigurator, GatewayConfigurator, VolumeConfigurator]


def configurator_for(conf_type: str):
    for c in CONFIGURATORS:
        if conf_type in c.TYPES:
            return c()
    raise ConfigurationError(f"unsupported configuration type {conf_type}")
