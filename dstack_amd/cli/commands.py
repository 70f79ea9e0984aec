"""``dstack`` sub-commands (reference: ``cli/commands/{apply,attach,config,delete,fleet,gateway,init,
logs,pool,ps,server,stats,stop,volume}.py``)."""

from __future__ import annotations

import argparse
import os
import sys
import time

from dstack_amd.cli.utils import (
    confirm_ask,
    console,
    fleets_table,
    gateways_table,
    print_table,
    runs_table,
    volumes_table,
)
from dstack_amd.core.errors import CLIError


def _client(args):
    from dstack_amd.api import Client

    return Client.from_config(project_name=getattr(args, "project", None))


def add_project_arg(p: argparse.ArgumentParser):
    p.add_argument("--project", metavar="NAME", help="Project name (default: the default project)")


# ---- server -----------------------------------------------------------------------------------
def register_server(sub):
    p = sub.add_parser("server", help="Start the dstack-amd server")
    p.add_argument("--host", default=os.getenv("DSTACK_SERVER_HOST", "127.0.0.1"))
    p.add_argument("-p", "--port", type=int, default=int(os.getenv("DSTACK_SERVER_PORT", "3000")))
    p.add_argument("-l", "--log-level", default=os.getenv("DSTACK_SERVER_LOG_LEVEL", "INFO"))
    p.add_argument("--token", default=os.getenv("DSTACK_SERVER_ADMIN_TOKEN"), help="Admin token")
    p.add_argument("-y", "--yes", action="store_true",
                   help="Make the server's project the CLI default without asking")
    p.add_argument("-n", "--no", action="store_true", help="Do not touch the CLI config")
    p.set_defaults(func=cmd_server)


def cmd_server(args) -> int:
    if args.yes:
        os.environ["DSTACK_UPDATE_DEFAULT_PROJECT"] = "1"
    if args.no:
        os.environ["DSTACK_DO_NOT_UPDATE_DEFAULT_PROJECT"] = "1"
    from dstack_amd.server import settings
    from dstack_amd.server.main import run

    settings.UPDATE_DEFAULT_PROJECT = settings.UPDATE_DEFAULT_PROJECT or args.yes
    settings.DO_NOT_UPDATE_DEFAULT_PROJECT = settings.DO_NOT_UPDATE_DEFAULT_PROJECT or args.no
    run(args.host, args.port, args.log_level, args.token)
    return 0


def _show(args, render) -> int:
    """Print ``render()`` once, or with ``--watch`` re-render it every second until Ctrl-C."""
    if not getattr(args, "watch", False):
        print_table(render())
        return 0
    from rich.live import Live

    try:
        with Live(render(), console=console, refresh_per_second=2) as live:
            while True:
                time.sleep(1)
                live.update(render())
    except KeyboardInterrupt:
        return 0


# ---- config / init ----------------------------------------------------------------------------
def register_config(sub):
    p = sub.add_parser("config", help="Configure a server project in ~/.dstack/config.yml")
    p.add_argument("--project", help="Project name")
    p.add_argument("--url", help="Server URL")
    p.add_argument("--token", help="User token")
    p.add_argument("--default", action="store_true", help="Make the project the default")
    p.add_argument("--remove", action="store_true", help="Remove the project configuration")
    p.add_argument("-y", "--yes", action="store_true")
    p.add_argument("-n", "--no", action="store_true")
    p.set_defaults(func=cmd_config)


def cmd_config(args) -> int:
    from dstack_amd.api.server import APIClient
    from dstack_amd.core.services.configs import ConfigManager

    cm = ConfigManager()
    if args.remove:
        if not args.project:
            raise CLIError("--project is required with --remove")
        if args.yes or confirm_ask(f"Remove the project [code]{args.project}[/] configuration?"):
            cm.delete_project(args.project)
            cm.save()
            console.print(f"Project [code]{args.project}[/] configuration removed")
        return 0
    if not (args.project and args.url and args.token):
        for p in cm.config.projects:
            console.print(f"{p.name}\t{p.url}{'  (default)' if p.default else ''}")
        if not cm.config.projects:
            console.print("No projects configured. Use: dstack config --url URL --project NAME --token TOKEN")
        return 0
    # validate the token against the server before saving
    api = APIClient(args.url, args.token)
    try:
        api.projects.get(args.project)
    except Exception as e:  # noqa: BLE001
        raise CLIError(f"Cannot access project {args.project} at {args.url}: {e}") from e
    default = args.default or not cm.config.projects
    if not default and not args.no and not args.yes:
        default = confirm_ask(f"Set [code]{args.project}[/] as the default project?", default=False)
    cm.configure_project(args.project, args.url, args.token, default=default)
    cm.save()
    console.print(f"Configuration updated at {cm.config_filepath}")
    return 0


def register_init(sub):
    p = sub.add_parser("init", help="Initialise the current directory as a repo for runs")
    add_project_arg(p)
    p.add_argument("-t", "--token", help="Git OAuth token for private repos")
    p.add_argument("--git-identity", dest="git_identity_file", help="SSH key for private git repos")
    p.add_argument("--ssh-identity", dest="ssh_identity_file", help="SSH key for dstack attach")
    p.add_argument("--local", action="store_true", help="Upload the working tree instead of using git")
    p.set_defaults(func=cmd_init)


def cmd_init(args) -> int:
    from dstack_amd.core.models.repos import LocalRepo, RemoteRepo, RepoError
    from dstack_amd.core.services.configs import ConfigManager

    client = _client(args)
    cwd = os.getcwd()
    repo = None
    if not args.local:
        try:
            repo = RemoteRepo(cwd)
        except RepoError:
            repo = None
    if repo is None:
        repo = LocalRepo(cwd)
    client.repos.init(repo, git_identity_file=args.git_identity_file, oauth_token=args.token)
    cm = ConfigManager()
    key = args.ssh_identity_file or str(cm.ensure_ssh_key())
    cm.save_repo_config(cwd, repo.repo_id, "local" if isinstance(repo, LocalRepo) else "remote", key)
    console.print("OK")
    return 0


# ---- apply / delete ---------------------------------------------------------------------------
def register_apply(sub):
    from dstack_amd.cli.configurators import RunConfigurator, register_repo_args

    p = sub.add_parser("apply", help="Apply a configuration (run, fleet, gateway, volume)")
    add_project_arg(p)
    p.add_argument("-f", "--file", dest="configuration_file", help="Configuration file (default: .dstack.yml)")
    p.add_argument("-y", "--yes", action="store_true", help="Do not ask for confirmation")
    p.add_argument("--force", action="store_true", help="Re-create the resource even if unchanged")
    p.add_argument("-d", "--detach", action="store_true", help="Exit right after submitting")
    register_repo_args(p)
    RunConfigurator.register_args(p)
    p.set_defaults(func=cmd_apply)


def cmd_apply(args) -> int:
    from dstack_amd.cli.configurators import configurator_for, find_default_configuration, load_configuration

    path = args.configuration_file or find_default_configuration(os.getcwd())
    if path is None:
        raise CLIError("No configuration file given (-f) and no .dstack.yml in the current directory")
    conf = load_configuration(path)
    client = _client(args)
    return configurator_for(conf.type).apply(client, conf, path, args)


def register_delete(sub):
    p = sub.add_parser("delete", help="Delete the resources of a configuration (fleet, gateway, volume)")
    add_project_arg(p)
    p.add_argument("-f", "--file", dest="configuration_file", required=True)
    p.add_argument("-y", "--yes", action="store_true")
    p.set_defaults(func=cmd_delete)


def cmd_delete(args) -> int:
    from dstack_amd.cli.configurators import configurator_for, load_configuration

    conf = load_configuration(args.configuration_file)
    if conf.type in ("task", "service", "dev-environment"):
        raise CLIError("Use `dstack stop` for runs")
    return configurator_for(conf.type).delete(_client(args), conf, args)


# ---- ps / logs / stop / attach / stats --------------------------------------------------------
def register_ps(sub):
    p = sub.add_parser("ps", help="List runs")
    add_project_arg(p)
    p.add_argument("-a", "--all", action="store_true", help="Show finished runs too")
    p.add_argument("-v", "--verbose", action="store_true")
    p.add_argument("-w", "--watch", action="store_true", help="Refresh every second")
    p.add_argument("-n", "--last", type=int, default=None, help="Show the last N runs")
    p.set_defaults(func=cmd_ps)


def cmd_ps(args) -> int:
    client = _client(args)

    def table():
        runs = [r.model for r in client.runs.list(all=args.all, limit=args.last or 100)]
        if not args.all and not runs:
            runs = [r.model for r in client.runs.list(all=True, limit=1)]
        return runs_table(runs, verbose=args.verbose)

    if not args.watch:
        print_table(table())
        return 0
    from rich.live import Live

    try:
        with Live(table(), console=console, refresh_per_second=2) as live:
            while True:
                time.sleep(1)
                live.update(table())
    except KeyboardInterrupt:
        return 0


def register_logs(sub):
    p = sub.add_parser("logs", help="Show run logs")
    add_project_arg(p)
    p.add_argument("run_name")
    p.add_argument("-d", "--diagnose", action="store_true", help="Show runner logs (diagnostics)")
    p.add_argument("-a", "--attach", action="store_true", help="Follow the logs")
    p.add_argument("--replica", type=int, default=0)
    p.add_argument("--job", type=int, default=0)
    p.add_argument("--ssh-identity", dest="ssh_identity_file")
    p.set_defaults(func=cmd_logs)


def cmd_logs(args) -> int:
    client = _client(args)
    run = client.runs.get(args.run_name)
    if run is None:
        raise CLIError(f"Run {args.run_name} not found")
    try:
        for chunk in run.logs(diagnose=args.diagnose, replica_num=args.replica, job_num=args.job,
                              follow=args.attach):
            sys.stdout.buffer.write(chunk)
            sys.stdout.flush()
    except KeyboardInterrupt:
        pass
    return 0


def register_stop(sub):
    p = sub.add_parser("stop", help="Stop a run")
    add_project_arg(p)
    p.add_argument("run_name")
    p.add_argument("-x", "--abort", action="store_true", help="Abort without graceful shutdown")
    p.add_argument("-y", "--yes", action="store_true")
    p.set_defaults(func=cmd_stop)


def cmd_stop(args) -> int:
    client = _client(args)
    run = client.runs.get(args.run_name)
    if run is None:
        raise CLIError(f"Run {args.run_name} not found")
    verb = "abort" if args.abort else "stop"
    if not args.yes and not confirm_ask(f"Are you sure you want to {verb} the run [code]{args.run_name}[/]?"):
        return 0
    run.stop(abort=args.abort)
    console.print(f"Run [code]{args.run_name}[/] {'aborted' if args.abort else 'is stopping'}")
    return 0


def register_attach(sub):
    p = sub.add_parser("attach", help="Attach to a run: forward ports, optionally stream logs")
    add_project_arg(p)
    p.add_argument("run_name")
    p.add_argument("--ssh-identity", dest="ssh_identity_file")
    p.add_argument("--logs", action="store_true", help="Stream the run logs")
    p.add_argument("--host", dest="bind_address", default="127.0.0.1", help="Local address to bind")
    p.add_argument("-p", "--port", action="append", default=[], dest="ports", metavar="LOCAL:CONTAINER")
    p.add_argument("--replica", type=int, default=0)
    p.add_argument("--job", type=int, default=0)
    p.set_defaults(func=cmd_attach)


def cmd_attach(args) -> int:
    client = _client(args)
    run = client.runs.get(args.run_name)
    if run is None:
        raise CLIError(f"Run {args.run_name} not found")
    overrides = {}
    for p in args.ports:
        local, _, container = p.partition(":")
        if not container:
            raise CLIError(f"invalid port mapping {p}: use LOCAL:CONTAINER")
        overrides[int(container)] = int(local)
    if not run.attach(ssh_identity_file=args.ssh_identity_file, bind_address=args.bind_address,
                      ports_overrides=overrides):
        raise CLIError(f"Run {args.run_name} is not running")
    for cport, lport in (run.ports or {}).items():
        console.print(f"Forwarded port {cport} -> {args.bind_address}:{lport}")
    try:
        if args.logs:
            for chunk in run.logs(follow=True):
                sys.stdout.buffer.write(chunk)
                sys.stdout.flush()
        else:
            console.print("Attached. Press Ctrl-C to detach.")
            while not run.refresh().status.is_finished():
                time.sleep(2)
    except KeyboardInterrupt:
        pass
    finally:
        run.detach()
    return 0


def register_stats(sub):
    p = sub.add_parser("stats", help="Show run resource metrics (CPU, memory, GPU)")
    add_project_arg(p)
    p.add_argument("run_name")
    p.add_argument("-w", "--watch", action="store_true")
    p.set_defaults(func=cmd_stats)


def cmd_stats(args) -> int:
    from rich.table import Table

    client = _client(args)
    run = client.runs.get(args.run_name)
    if run is None:
        raise CLIError(f"Run {args.run_name} not found")

    def table():
        t = Table(box=None, header_style="bold")
        for col in ("NAME", "CPU", "MEMORY", "GPU"):
            t.add_column(col)
        for job in run.refresh().model.jobs:
            m = client.api.metrics.get_job_metrics(client.project, args.run_name, job.job_spec.replica_num,
                                                  job.job_spec.job_num)
            vals = {x.name: (x.values[-1] if x.values else None) for x in m.metrics}
            cpu = vals.get("cpu_usage_percent")
            mem = vals.get("memory_working_set_bytes")
            mem_total = vals.get("memory_total_bytes")
            gpus = []
            for i in range(int(vals.get("gpus_detected_num") or 0)):
                util, used = vals.get(f"gpu_util_percent_gpu{i}"), vals.get(f"gpu_memory_usage_bytes_gpu{i}")
                line = f"#{i} {_gb(used)} {util if util is not None else '-'}% util"
                power, hbm = vals.get(f"gpu_power_watts_gpu{i}"), vals.get(f"gpu_hbm_activity_percent_gpu{i}")
                if power is not None:
                    line += f" {power:.0f}W"
                if hbm is not None:
                    line += f" HBM {hbm:.0f}%"
                rd, wr = vals.get(f"gpu_xgmi_read_bytes_per_s_gpu{i}"), vals.get(f"gpu_xgmi_write_bytes_per_s_gpu{i}")
                if rd is not None or wr is not None:
                    line += f" xGMI rd {(rd or 0) / 1e9:.1f} wr {(wr or 0) / 1e9:.1f} GB/s"
                up = vals.get(f"gpu_xgmi_links_up_gpu{i}")
                if up is not None:
                    line += f" ({up:.0f} links up)"
                gpus.append(line)
            t.add_row(job.job_spec.job_name, f"{cpu}%" if cpu is not None else "-",
                      f"{_gb(mem)}/{_gb(mem_total)}" if mem_total else _gb(mem), "\n".join(gpus) or "-")
        return t

    if not args.watch:
        print_table(table())
        return 0
    from rich.live import Live

    try:
        with Live(table(), console=console, refresh_per_second=1) as live:
            while True:
                time.sleep(2)
                live.update(table())
    except KeyboardInterrupt:
        return 0


def _gb(v) -> str:
    return "-" if v is None else f"{v / 2**30:.1f}GB"


# ---- offer ------------------------------------------------------------------------------------
def register_offer(sub):
    p = sub.add_parser("offer", help="List the offers of every configured backend for a resource spec "
                                     "(live provider listings where the backend has one)")
    add_project_arg(p)
    p.add_argument("--gpu", metavar="SPEC", help="GPU spec, e.g. MI355X:8, 192GB..:1.., amd:8")
    p.add_argument("--cpu", metavar="SPEC")
    p.add_argument("--memory", metavar="SPEC")
    p.add_argument("--disk", metavar="SPEC")
    g = p.add_mutually_exclusive_group()
    g.add_argument("--spot", dest="spot_policy", action="store_const", const="spot")
    g.add_argument("--on-demand", dest="spot_policy", action="store_const", const="on-demand")
    p.add_argument("--max-price", type=float)
    p.add_argument("-b", "--backend", action="append", dest="backends", metavar="NAME")
    p.add_argument("-r", "--region", action="append", dest="regions", metavar="NAME")
    p.add_argument("-n", "--max-offers", type=int, default=50)
    p.add_argument("--json", action="store_true", help="print the offers as JSON")
    p.set_defaults(func=cmd_offer)


def cmd_offer(args) -> int:
    import json

    from rich.table import Table

    from dstack_amd.core.models.configurations import parse_run_configuration

    resources = {k: getattr(args, k) for k in ("gpu", "cpu", "memory", "disk") if getattr(args, k)}
    conf = {"type": "task", "commands": [":"], "resources": resources, "spot_policy": args.spot_policy or "auto"}
    for k, v in (("max_price", args.max_price), ("backends", args.backends), ("regions", args.regions)):
        if v:
            conf[k] = v
    client = _client(args)
    plan = client.runs.get_plan(parse_run_configuration(conf), max_offers=args.max_offers)
    jp = plan.job_plans[0]
    if args.json:
        print(json.dumps({"total_offers": jp.total_offers, "max_price": jp.max_price,
                          "offers": [o.model_dump(mode="json") for o in jp.offers]}, indent=1))
        return 0
    t = Table(box=None, header_style="bold")
    for col in ("#", "BACKEND", "REGION", "INSTANCE", "RESOURCES", "SPOT", "PRICE", "AVAILABILITY"):
        t.add_column(col, no_wrap=col != "RESOURCES")
    for i, o in enumerate(jp.offers, 1):
        r = o.instance.resources
        t.add_row(str(i), o.backend.value, o.region, o.instance.name, r.pretty_format(), "yes" if r.spot else "no",
                  f"${o.price:.4g}", o.availability.value)
    print_table(t)
    console.print(f"{len(jp.offers)} of {jp.total_offers} offers shown"
                  + (f", up to ${jp.max_price:.4g}/h" if jp.max_price is not None else ""))
    return 0


# ---- fleet / volume / gateway / pool ----------------------------------------------------------
def register_fleet(sub):
    p = sub.add_parser("fleet", help="Manage fleets")
    add_project_arg(p)
    p.add_argument("-v", "--verbose", action="store_true")
    p.add_argument("-w", "--watch", action="store_true", help="Update listing in realtime")
    p.set_defaults(func=cmd_fleet_list)
    s = p.add_subparsers(dest="fleet_cmd")
    lp = s.add_parser("list")
    lp.add_argument("-v", "--verbose", action="store_true")
    lp.add_argument("-w", "--watch", action="store_true", help="Update listing in realtime")
    add_project_arg(lp)
    lp.set_defaults(func=cmd_fleet_list)
    dp = s.add_parser("delete")
    add_project_arg(dp)
    dp.add_argument("name")
    dp.add_argument("-i", "--instance", type=int, action="append", dest="instance_nums")
    dp.add_argument("-y", "--yes", action="store_true")
    dp.set_defaults(func=cmd_fleet_delete)


def cmd_fleet_list(args) -> int:
    client = _client(args)
    return _show(args, lambda: fleets_table(client.api.fleets.list(client.project),
                                            verbose=getattr(args, "verbose", False)))


def cmd_fleet_delete(args) -> int:
    client = _client(args)
    if args.instance_nums:
        if args.yes or confirm_ask(f"Delete instances {args.instance_nums} of fleet [code]{args.name}[/]?"):
            client.api.fleets.delete_instances(client.project, args.name, args.instance_nums)
            console.print("Instances deleted")
        return 0
    if args.yes or confirm_ask(f"Delete the fleet [code]{args.name}[/]?"):
        client.api.fleets.delete(client.project, [args.name])
        console.print(f"Fleet [code]{args.name}[/] deleted")
    return 0


def register_volume(sub):
    p = sub.add_parser("volume", help="Manage volumes")
    add_project_arg(p)
    p.add_argument("-w", "--watch", action="store_true", help="Update listing in realtime")
    p.set_defaults(func=cmd_volume_list, verbose=False)
    s = p.add_subparsers(dest="volume_cmd")
    lp = s.add_parser("list")
    add_project_arg(lp)
    lp.add_argument("-v", "--verbose", action="store_true")
    lp.add_argument("-w", "--watch", action="store_true", help="Update listing in realtime")
    lp.set_defaults(func=cmd_volume_list)
    dp = s.add_parser("delete")
    add_project_arg(dp)
    dp.add_argument("name")
    dp.add_argument("-y", "--yes", action="store_true")
    dp.set_defaults(func=cmd_volume_delete)


def cmd_volume_list(args) -> int:
    client = _client(args)
    return _show(args, lambda: volumes_table(client.api.volumes.list(client.project)))


def cmd_volume_delete(args) -> int:
    client = _client(args)
    if args.yes or confirm_ask(f"Delete the volume [code]{args.name}[/]?"):
        client.api.volumes.delete(client.project, [args.name])
        console.print(f"Volume [code]{args.name}[/] deleted")
    return 0


def register_gateway(sub):
    p = sub.add_parser("gateway", help="Manage gateways")
    add_project_arg(p)
    p.add_argument("-w", "--watch", action="store_true", help="Update listing in realtime")
    p.set_defaults(func=cmd_gateway_list)
    s = p.add_subparsers(dest="gateway_cmd")
    lp = s.add_parser("list")
    add_project_arg(lp)
    lp.add_argument("-v", "--verbose", action="store_true")
    lp.add_argument("-w", "--watch", action="store_true", help="Update listing in realtime")
    lp.set_defaults(func=cmd_gateway_list)
    cp = s.add_parser("create")
    add_project_arg(cp)
    cp.add_argument("--backend", required=True)
    cp.add_argument("--region", required=True)
    cp.add_argument("--set-default", action="store_true")
    cp.add_argument("--name")
    cp.add_argument("--domain", required=True)
    cp.set_defaults(func=cmd_gateway_create)
    dp = s.add_parser("delete")
    add_project_arg(dp)
    dp.add_argument("name")
    dp.add_argument("-y", "--yes", action="store_true")
    dp.set_defaults(func=cmd_gateway_delete)
    up = s.add_parser("update")
    add_project_arg(up)
    up.add_argument("name")
    up.add_argument("--set-default", action="store_true")
    up.add_argument("--domain")
    up.set_defaults(func=cmd_gateway_update)


def cmd_gateway_list(args) -> int:
    client = _client(args)
    return _show(args, lambda: gateways_table(client.api.gateways.list(client.project)))


def cmd_gateway_create(args) -> int:
    from dstack_amd.core.models.gateways import GatewayConfiguration

    client = _client(args)
    conf = GatewayConfiguration(name=args.name, backend=args.backend, region=args.region, domain=args.domain,
                                default=args.set_default)
    gw = client.api.gateways.create(client.project, conf)
    print_table(gateways_table([gw]))
    return 0


def cmd_gateway_delete(args) -> int:
    client = _client(args)
    if args.yes or confirm_ask(f"Delete the gateway [code]{args.name}[/]?"):
        client.api.gateways.delete(client.project, [args.name])
        console.print(f"Gateway [code]{args.name}[/] deleted")
    return 0


def cmd_gateway_update(args) -> int:
    client = _client(args)
    if args.set_default:
        client.api.gateways.set_default(client.project, args.name)
    if args.domain is not None:
        client.api.gateways.set_wildcard_domain(client.project, args.name, args.domain)
    print_table(gateways_table([client.api.gateways.get(client.project, args.name)]))
    return 0


def register_pool(sub):
    """``dstack pool`` (reference: cli/commands/pool.py; deprecated there in favour of fleets)."""
    p = sub.add_parser("pool", help="(Deprecated: use fleets) manage pools and pool instances")
    add_project_arg(p)
    s = p.add_subparsers(dest="pool_cmd")
    lp = s.add_parser("list", help="List pools")
    lp.add_argument("-v", "--verbose", action="store_true")
    lp.set_defaults(func=cmd_pool_list)
    cp = s.add_parser("create", help="Create a pool")
    cp.add_argument("-n", "--name", dest="pool_name", required=True)
    cp.set_defaults(func=cmd_pool_create)
    dp = s.add_parser("delete", help="Delete a pool")
    dp.add_argument("-n", "--name", dest="pool_name", required=True)
    dp.set_defaults(func=cmd_pool_delete)
    pp = s.add_parser("ps", help="Show pool instances")
    pp.add_argument("--pool", dest="pool_name")
    pp.add_argument("-w", "--watch", action="store_true")
    pp.set_defaults(func=cmd_pool_ps)
    ap = s.add_parser("add", help="Add a cloud instance to the pool")
    ap.add_argument("-y", "--yes", action="store_true")
    ap.add_argument("--max-offers", type=int, default=3)
    ap.add_argument("--gpu", help="GPU requirement, e.g. MI355X:8")
    ap.add_argument("--cpu", help="CPU requirement, e.g. 32..")
    ap.add_argument("--memory", help="Memory requirement, e.g. 256GB..")
    ap.add_argument("--disk", help="Disk requirement, e.g. 500GB..")
    ap.add_argument("--shared-memory", dest="shared_memory", metavar="SIZE", help="Shared memory size, e.g. 64GB")
    ap.add_argument("--pool", dest="pool_name")
    ap.add_argument("--max-price", type=float)
    ap.add_argument("-b", "--backend", action="append", dest="backends")
    ap.add_argument("-r", "--region", action="append", dest="regions")
    ap.add_argument("--spot-policy", dest="spot_policy")
    ap.set_defaults(func=cmd_pool_add)
    rp = s.add_parser("rm", aliases=["remove"], help="Remove an instance from the pool")
    rp.add_argument("instance_name")
    rp.add_argument("--pool", dest="pool_name")
    rp.add_argument("--force", action="store_true")
    rp.add_argument("-y", "--yes", action="store_true")
    rp.set_defaults(func=cmd_pool_rm)
    sp = s.add_parser("set-default", help="Set the project's default pool")
    sp.add_argument("--pool", dest="pool_name", required=True)
    sp.set_defaults(func=cmd_pool_set_default)
    hp = s.add_parser("add-ssh", help="Add an SSH host (e.g. an on-prem MI355X node) to the pool")
    hp.add_argument("destination", help="[user@]host")
    hp.add_argument("-i", dest="ssh_identity_file", required=True, metavar="SSH_PRIVATE_KEY")
    hp.add_argument("-p", dest="ssh_port", type=int)
    hp.add_argument("-l", dest="login_name")
    hp.add_argument("--region")
    hp.add_argument("--pool", dest="pool_name")
    hp.add_argument("--name", dest="instance_name")
    hp.add_argument("--network", help="Network for multinode setups, <ip>/<mask>")
    hp.set_defaults(func=cmd_pool_add_ssh)
    p.set_defaults(func=cmd_pool_ps, pool_name=None, watch=False)


def _instances_table(instances):
    from rich.table import Table

    from dstack_amd.cli.utils import pretty_date

    t = Table(box=None, header_style="bold")
    for col in ("INSTANCE", "BACKEND", "RESOURCES", "PRICE", "STATUS", "CREATED"):
        t.add_column(col)
    for inst in instances:
        t.add_row(inst.name, f"{inst.backend.value if inst.backend else ''} ({inst.region or ''})",
                  inst.instance_type.resources.pretty_format() if inst.instance_type else "",
                  f"${inst.price:.4g}" if inst.price is not None else "", inst.status.value, pretty_date(inst.created))
    return t


def cmd_pool_list(args) -> int:
    from rich.table import Table

    from dstack_amd.cli.utils import pretty_date

    client = _client(args)
    t = Table(box=None, header_style="bold")
    for col in ("NAME", "DEFAULT", "INSTANCES", "AVAILABLE", "CREATED"):
        t.add_column(col)
    for pool in client.api.pool.list(client.project):
        t.add_row(pool.name, "yes" if pool.default else "", str(pool.total_instances), str(pool.available_instances),
                  pretty_date(pool.created_at))
    print_table(t)
    return 0


def cmd_pool_create(args) -> int:
    client = _client(args)
    client.api.pool.create(client.project, args.pool_name)
    console.print(f"Pool {args.pool_name!r} created")
    return 0


def cmd_pool_delete(args) -> int:
    client = _client(args)
    client.api.pool.delete(client.project, args.pool_name, False)
    console.print(f"Pool {args.pool_name!r} removed")
    return 0


def cmd_pool_ps(args) -> int:
    import time

    client = _client(args)
    while True:
        pool = client.api.pool.show(client.project, args.pool_name)
        console.print(f" Pool name  {pool.name}\n")
        print_table(_instances_table(pool.instances))
        if not args.watch:
            return 0
        time.sleep(2)


def cmd_pool_rm(args) -> int:
    client = _client(args)
    pool = client.api.pool.show(client.project, args.pool_name)
    if not any(i.name == args.instance_name for i in pool.instances):
        raise CLIError(f"Instance {args.instance_name!r} not found in pool {pool.name!r}")
    if args.yes or confirm_ask(f"Remove instance [code]{args.instance_name}[/]?"):
        client.api.pool.remove(client.project, pool.name, args.instance_name, args.force)
        console.print(f"Instance {args.instance_name!r} removed")
    return 0


def cmd_pool_set_default(args) -> int:
    client = _client(args)
    client.api.pool.set_default(client.project, args.pool_name)
    return 0


def _pool_requirements(args):
    from dstack_amd.core.models.profiles import Profile, SpotPolicy
    from dstack_amd.core.models.resources import ResourcesSpec
    from dstack_amd.core.models.runs import Requirements, get_policy_map

    res = {}
    for k in ("gpu", "cpu", "memory", "disk"):
        if getattr(args, k, None):
            res[k] = getattr(args, k)
    if getattr(args, "shared_memory", None):
        res["shm_size"] = args.shared_memory
    spot = SpotPolicy(args.spot_policy) if args.spot_policy else None
    profile = Profile(name="pool-add", backends=args.backends, regions=args.regions, max_price=args.max_price,
                      spot_policy=spot, pool_name=args.pool_name)
    req = Requirements(resources=ResourcesSpec.model_validate(res), max_price=args.max_price,
                       spot=get_policy_map(spot, SpotPolicy.ONDEMAND))
    return profile, req


def cmd_pool_add(args) -> int:
    from rich.table import Table

    client = _client(args)
    profile, req = _pool_requirements(args)
    offers = client.api.pool.get_offers(client.project, profile, req)
    if not offers.instances:
        raise CLIError("No offers match the requirements")
    t = Table(box=None, header_style="bold")
    for col in ("#", "BACKEND", "REGION", "INSTANCE", "RESOURCES", "PRICE"):
        t.add_column(col)
    for i, o in enumerate(offers.instances[: args.max_offers], 1):
        t.add_row(str(i), o.backend.value, o.region, o.instance.name, o.instance.resources.pretty_format(),
                  f"${o.price:.4g}")
    print_table(t)
    if not (args.yes or confirm_ask(f"Add an instance to pool [code]{offers.pool_name}[/]?")):
        return 0
    inst = client.api.pool.create_instance(client.project, profile, req)
    print_table(_instances_table([inst]))
    return 0


def cmd_pool_add_ssh(args) -> int:
    from dstack_amd.core.models.instances import SSHKey

    client = _client(args)
    user, _, host = args.destination.rpartition("@")
    user = args.login_name or user or "root"
    key_path = os.path.expanduser(args.ssh_identity_file)
    with open(key_path) as f:
        private = f.read()
    public = ""
    if os.path.exists(key_path + ".pub"):
        with open(key_path + ".pub") as f:
            public = f.read().strip()
    inst = client.api.pool.add_remote(client.project, host=host, port=args.ssh_port or 22, ssh_user=user,
                                      ssh_keys=[SSHKey(public=public, private=private)], pool_name=args.pool_name,
                                      instance_name=args.instance_name, region=args.region,
                                      instance_network=args.network)
    print_table(_instances_table([inst]))
    return 0


# ---- run (deprecated alias of apply for run configurations; reference cli/commands/run.py) ------
def register_run(sub):
    from dstack_amd.cli.configurators import RunConfigurator, register_repo_args

    p = sub.add_parser("run", help="(Deprecated: use apply) run a configuration")
    add_project_arg(p)
    p.add_argument("working_dir")
    p.add_argument("-f", "--file", dest="configuration_file", help="Configuration file (default: .dstack.yml)")
    p.add_argument("-y", "--yes", action="store_true", help="Do not ask for confirmation")
    p.add_argument("-d", "--detach", action="store_true", help="Exit right after submitting")
    p.add_argument("--force", action="store_true", help=argparse.SUPPRESS)
    register_repo_args(p)
    RunConfigurator.register_args(p)
    p.set_defaults(func=cmd_run)


def cmd_run(args) -> int:
    from dstack_amd.cli.configurators import configurator_for, find_default_configuration, load_configuration

    console.print("[yellow]dstack run is deprecated in favor of dstack apply[/]")
    base = os.path.abspath(args.working_dir)
    path = args.configuration_file or find_default_configuration(base)
    if path is None:
        raise CLIError(f"No configuration file given (-f) and no .dstack.yml in {base}")
    conf = load_configuration(path)
    if conf.type not in ("task", "service", "dev-environment"):
        raise CLIError(f"dstack run only runs task/service/dev-environment configurations, got {conf.type}")
    if getattr(args, "repo", None) is None:
        args.repo = base
    client = _client(args)
    return configurator_for(conf.type).apply(client, conf, path, args)


REGISTRARS = [register_server, register_config, register_init, register_apply, register_delete, register_ps,
              register_logs, register_stop, register_attach, register_stats, register_offer, register_fleet,
              register_volume, register_gateway, register_pool, register_run]
