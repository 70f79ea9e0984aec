"""CLI rendering helpers (reference: ``cli/utils/{common,run,fleet,volume,gateway}.py``): rich tables
for runs, offers, fleets, volumes and gateways, confirm prompts, and the run-status colours."""

from __future__ import annotations

import sys
from datetime import datetime, timezone
from typing import Iterable, Optional

from rich.console import Console
from rich.table import Table

from dstack_amd.core.models.runs import Run, RunPlan, RunStatus

console = Console(highlight=False)
err_console = Console(stderr=True, highlight=False)

_STATUS_STYLE = {
    "submitted": "grey58", "pending": "grey58", "provisioning": "deep_sky_blue1", "pulling": "sea_green3",
    "running": "sea_green3", "terminating": "deep_sky_blue1", "terminated": "grey58", "aborted": "grey58",
    "failed": "indian_red1", "done": "grey58",
}


def confirm_ask(prompt: str, default: bool = True) -> bool:
    if not sys.stdin.isatty():
        return default
    suffix = " [Y/n]: " if default else " [y/N]: "
    try:
        ans = input(prompt + suffix).strip().lower()
    except EOFError:
        return default
    if not ans:
        return default
    return ans in ("y", "yes")


def pretty_date(dt: Optional[datetime]) -> str:
    from dstack_amd.utils.common import pretty_date as _pretty

    return _pretty(dt)


def status_text(status: str, error: Optional[str] = None, exit_status: Optional[int] = None) -> str:
    style = _STATUS_STYLE.get(status, "white")
    s = status
    if status == "failed" and exit_status not in (None, 0):
        s = f"exited ({exit_status})"
    elif error and status in ("failed", "terminated"):
        s = f"{status} ({error.lower()})"
    return f"[{style}]{s}[/]"


def runs_table(runs: Iterable[Run], verbose: bool = False) -> Table:
    t = Table(box=None, header_style="bold", pad_edge=False)
    for col in ("NAME", "BACKEND", "RESOURCES", "PRICE", "STATUS", "SUBMITTED"):
        t.add_column(col, no_wrap=col != "RESOURCES")
    if verbose:
        t.add_column("ERROR")
    for run in runs:
        multi = len(run.jobs) > 1
        t.add_row(f"[bold]{run.run_spec.run_name}[/]", "" if multi else _backend(run.jobs[0] if run.jobs else None),
                  "" if multi else _resources(run.jobs[0] if run.jobs else None),
                  "" if multi else _price(run.jobs[0] if run.jobs else None),
                  status_text(run.status.value, run.error), pretty_date(run.submitted_at), *([run.error or ""] if verbose else []))
        if multi:
            for job in run.jobs:
                sub = job.job_submissions[-1]
                name = f"  replica={job.job_spec.replica_num} job={job.job_spec.job_num}"
                t.add_row(name, _backend(job), _resources(job), _price(job),
                          status_text(sub.status.value, sub.termination_reason.name if sub.termination_reason else None,
                                      sub.exit_status), pretty_date(sub.submitted_at),
                          *([sub.termination_reason_message or ""] if verbose else []))
    return t


def _backend(job) -> str:
    if job is None or not job.job_submissions:
        return ""
    jpd = job.job_submissions[-1].job_provisioning_data
    if jpd is None:
        return ""
    return f"{jpd.backend.value} ({jpd.region})"


def _resources(job) -> str:
    if job is None or not job.job_submissions:
        return ""
    jpd = job.job_submissions[-1].job_provisioning_data
    if jpd is None:
        return ""
    s = jpd.instance_type.resources.pretty_format()
    jrd = job.job_submissions[-1].job_runtime_data
    if jrd is not None and jrd.gpu_indices:
        s += f" gpus={','.join(map(str, jrd.gpu_indices))}"
    return s


def _price(job) -> str:
    if job is None or not job.job_submissions:
        return ""
    jpd = job.job_submissions[-1].job_provisioning_data
    return f"${jpd.price:.4g}" if jpd is not None else ""


def plan_table(plan: RunPlan, max_offers: int = 3) -> Table:
    job_plan = plan.job_plans[0]
    spec = job_plan.job_spec
    prof = plan.run_spec.merged_profile
    props = Table(box=None, show_header=False)
    props.add_column(no_wrap=True)
    props.add_column()
    conf = plan.run_spec.configuration
    props.add_row("[bold]Project[/]", plan.project_name)
    props.add_row("[bold]User[/]", plan.user)
    props.add_row("[bold]Configuration[/]", plan.run_spec.configuration_path or "-")
    props.add_row("[bold]Type[/]", conf.type)
    props.add_row("[bold]Resources[/]", spec.requirements.resources.pretty_format())
    if getattr(conf, "nodes", 1) and getattr(conf, "nodes", 1) > 1:
        props.add_row("[bold]Nodes[/]", str(conf.nodes))
    props.add_row("[bold]Max price[/]", f"${prof.max_price:g}" if prof.max_price else "-")
    props.add_row("[bold]Max duration[/]", str(spec.max_duration or "-"))
    props.add_row("[bold]Spot policy[/]", (prof.spot_policy.value if prof.spot_policy else "auto"))
    props.add_row("[bold]Retry policy[/]", "yes" if prof.retry else "no")
    props.add_row("[bold]Creation policy[/]", prof.creation_policy.value if prof.creation_policy else "-")
    props.add_row("[bold]Idle duration[/]", str(prof.idle_duration) if prof.idle_duration is not None else "-")
    offers = Table(box=None, header_style="bold")
    for col in ("#", "BACKEND", "REGION", "INSTANCE", "RESOURCES", "SPOT", "PRICE", ""):
        offers.add_column(col, no_wrap=col != "RESOURCES")
    for i, o in enumerate(job_plan.offers[:max_offers], 1):
        r = o.instance.resources
        avail = "" if o.availability.value in ("available", "unknown") else o.availability.value
        if o.total_blocks > 1:
            avail = f"{o.blocks}/{o.total_blocks} blocks " + avail
        offers.add_row(str(i), o.backend.value, o.region, o.instance.name, r.pretty_format(),
                       "yes" if r.spot else "no", f"${o.price:.4g}", avail)
    if job_plan.total_offers > max_offers:
        offers.add_row("", "...", "", "", "", "", "", f"shown {max_offers} of {job_plan.total_offers} offers")
    outer = Table(box=None, show_header=False)
    outer.add_column()
    outer.add_row(props)
    outer.add_row("")
    outer.add_row(offers)
    return outer


def fleets_table(fleets, verbose: bool = False) -> Table:
    t = Table(box=None, header_style="bold")
    cols = ["FLEET", "INSTANCE", "BACKEND", "RESOURCES", "PRICE", "STATUS", "CREATED"]
    if verbose:
        cols.append("GPU HEALTH")  # the HIP probe: HBM TB/s, bf16 MFMA TF/s, xGMI / RCCL GB/s
    for col in cols:
        t.add_column(col, no_wrap=col != "RESOURCES")
    for f in fleets:
        if not f.instances:
            t.add_row(f.name, "", "", "", "", f.status.value, pretty_date(f.created_at), *([""] if verbose else []))
        for i, inst in enumerate(f.instances):
            res = inst.instance_type.resources.pretty_format() if inst.instance_type else ""
            st = inst.status.value + (" (unreachable)" if inst.unreachable else "")
            if inst.total_blocks and inst.total_blocks > 1:
                st += f" {inst.busy_blocks}/{inst.total_blocks} busy"
            row = [f.name if i == 0 else "", str(inst.instance_num),
                   f"{inst.backend.value if inst.backend else ''} ({inst.region or ''})", res,
                   f"${inst.price:.4g}" if inst.price is not None else "", st, pretty_date(inst.created)]
            if verbose:
                row.append(health_summary(inst.health))
            t.add_row(*row)
    return t


def health_summary(h) -> str:
    if not h:
        return "-"
    parts = ["ok" if h.get("healthy", True) else f"[red]{h.get('message') or 'unhealthy'}[/]"]
    for key, unit in (("hbm_tb_s", "TB/s HBM"), ("mfma_bf16_tflops", "TF/s bf16"), ("xgmi_gb_s", "GB/s xGMI"),
                      ("rccl_busbw_gb_s", "GB/s RCCL")):
        if h.get(key):
            parts.append(f"{float(h[key]):.4g} {unit}")
    return ", ".join(parts)


def volumes_table(volumes, verbose: bool = False) -> Table:
    t = Table(box=None, header_style="bold")
    for col in ("NAME", "BACKEND", "REGION", "STATUS", "CREATED"):
        t.add_column(col)
    for v in volumes:
        t.add_row(v.name, v.configuration.backend.value, v.configuration.region or "", v.status.value,
                  pretty_date(v.created_at))
    return t


def gateways_table(gateways, verbose: bool = False) -> Table:
    t = Table(box=None, header_style="bold")
    for col in ("NAME", "BACKEND", "REGION", "HOSTNAME", "DOMAIN", "DEFAULT", "STATUS"):
        t.add_column(col)
    for g in gateways:
        t.add_row(g.name, g.backend.value if g.backend else "", g.region or "", g.hostname or "",
                  g.wildcard_domain or "", "✓" if g.default else "", g.status.value)
    return t


def print_table(t: Table):
    console.print(t)
    console.print()
