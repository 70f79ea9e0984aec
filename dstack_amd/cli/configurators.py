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
from dstack_amd.core.models.configurations import PortMapping, ServiceConfiguration
from dstack_amd.core.models.envs import Env
from dstack_amd.core.models.profiles import CreationPolicy, Profile, ProfilesConfig, SpotPolicy, TerminationPolicy
from dstack_amd.core.models.repos import LocalRepo, RemoteRepo, Repo, RepoError, VirtualRepo
from dstack_amd.core.models.runs import JobStatus, RunStatus


# ---- profile arguments (cli/services/profile.py) ----------------------------------------------
def register_profile_args(parser: argparse.ArgumentParser):
    g = parser.add_argument_group("Profile")
    g.add_argument("--profile", metavar="NAME", help="Profile from .dstack/profiles.yml")
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


def load_profile(repo_dir: str, name: Optional[str]) -> Optional[Profile]:
    path = Path(repo_dir) / ".dstack" / "profiles.yml"
    if not path.exists():
        if name:
            raise CLIError(f"profile {name} not found: {path} does not exist")
        return None
    cfg = ProfilesConfig.model_validate(yaml.safe_load(path.read_text()) or {"profiles": []})
    if name:
        for p in cfg.profiles:
            if p.name == name:
                return p
        raise CLIError(f"profile {name} not found in {path}")
    return cfg.default()


def apply_profile_args(args, profile: Profile):
    if args.max_price is not None:
        profile.max_price = args.max_price
    if args.max_duration is not None:
        profile.max_duration = args.max_duration
    if args.backends:
        profile.backends = args.backends
    if args.regions:
        profile.regions = args.regions
    if args.instance_types:
        profile.instance_types = args.instance_types
    if args.pool_name:
        profile.pool_name = args.pool_name
    if args.creation_policy_reuse:
        profile.creation_policy = CreationPolicy.REUSE
    if args.dont_destroy:
        profile.termination_policy = TerminationPolicy.DONT_DESTROY
    if args.idle_duration is not None:
        profile.idle_duration = args.idle_duration
    if args.instance_name:
        profile.instance_name = args.instance_name
        profile.creation_policy = CreationPolicy.REUSE
    if args.spot_policy is not None:
        profile.spot_policy = args.spot_policy
    if args.retry_policy is not None:
        if args.retry_policy:
            profile.retry = {"on_events": ["no-capacity", "interruption", "error"],
                             "duration": args.retry_duration}
        else:
            profile.retry = False
    elif args.retry_duration:
        profile.retry = {"on_events": ["no-capacity", "interruption", "error"], "duration": args.retry_duration}


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

    def apply(self, client: Client, conf, conf_path: str, args) -> int:
        if args.env:
            env = Env(conf.env)
            for e in args.env:
                if "=" in e:
                    k, v = e.split("=", 1)
                    env[k] = v
                elif e in os.environ:
                    env[e] = os.environ[e]
                else:
                    raise CLIError(f"{e} is not set in the local environment")
            conf.env = env
        try:  # `env: [HF_TOKEN]` takes the value from the local environment
            conf.env = Env(conf.env).resolve(os.environ)
        except (KeyError, ValueError) as e:
            raise CLIError(f"Environment variable not set locally: {e}") from e
        if args.gpu:
            conf.resources.gpu = args.gpu
            conf.resources = type(conf.resources).model_validate(conf.resources.model_dump())
        if args.disk:
            conf.resources.disk = args.disk
            conf.resources = type(conf.resources).model_validate(conf.resources.model_dump())
        if args.ports and hasattr(conf, "ports"):
            conf.ports = list(conf.ports) + [PortMapping.parse(p) for p in args.ports]
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
        pass

    def apply(self, client: Client, conf, conf_path: str, args) -> int:
        from dstack_amd.core.models.fleets import FleetSpec

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


_ = (ServiceConfiguration, Dict, List)
