"""The headline metric literally: ``examples/llama3-8b-train`` applied through the server.

A real dstack-amd server (local backend: native ``dstack-shim`` process driver + ``dstack-runner``,
one freshly started agent per instance) receives the example task through the public API (what
``dstack apply -f examples/llama3-8b-train/train.dstack.yml`` does), with ``MI355X:N`` when the host
has GPUs.  The task's own commands run: the extension build check, then ``torchrun ... bench.py``
(N ranks, RCCL), whose rank 0 prints its start-up stages (``[train] stages``, wall clock) after the
first optimizer step and its tokens/s result line at the end.

Reported (one JSON line):

* ``time_to_first_step_p50_s``: submit -> the task's first optimizer step finished, p50 over
  ``--runs`` runs that each land on a NEW instance (the previous one is retired first), with the
  stage split: control plane (offer, instance, agent, runner start), launch (the task's shell,
  build check, torchrun, interpreter exec), imports, rendezvous, extension load, GEMM selections,
  model init and the first step itself;
* ``job_tokens_per_s``: the tokens/s the task itself printed (its own timed steps), from a final
  run with ``--tok-steps`` timed steps.

Not included (local backend): VM boot, image pull, container start.
"""

from __future__ import annotations

import argparse
import json
import os
import re
import statistics
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
EXAMPLE = os.path.join(REPO, "examples", "llama3-8b-train", "train.dstack.yml")
# the launcher env of an enclosing torchrun must not leak into the server and its jobs
_LAUNCHER_ENV = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
                 "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT",
                 "TORCHELASTIC_RESTART_COUNT", "TORCHELASTIC_MAX_RESTARTS", "TORCHELASTIC_RUN_ID",
                 "TORCHELASTIC_USE_AGENT_STORE", "TORCHELASTIC_ERROR_FILE", "TORCH_NCCL_ASYNC_ERROR_HANDLING",
                 "DSTACK_AMD_BENCH_CHILD")

STAGES = [  # (name, start stamp, end stamp) -- stamps: server timings + the task's [train] stages
    # "running": the server has handed the job to the runner; "proc_start": rank 0's exec
    ("control_plane_s", "submitted", "running"),
    ("launch_s", "running", "proc_start"),
    ("imports_s", "proc_start", "torch_imported"),
    ("rendezvous_s", "torch_imported", "dist_ready"),
    ("extension_load_s", "dist_ready", "extension_loaded"),
    ("gemm_tuning_s", "extension_loaded", "gemm_tuning_loaded"),
    ("model_init_s", "gemm_tuning_loaded", "model_ready"),
    ("first_step_s", "model_ready", "first_step_done"),
]


def _free_port_pair() -> int:
    """A port p with p and p + 1 free on this host (the task's store and its RCCL pre-flight)."""
    import socket

    for _ in range(50):
        with socket.socket() as a:
            a.bind(("127.0.0.1", 0))
            port = a.getsockname()[1]
            if port >= 65535:
                continue
            with socket.socket() as b:
                try:
                    b.bind(("127.0.0.1", port + 1))
                except OSError:
                    continue
            return port
    return 29611


def task_conf(gpus: int, steps: int, warmup: int, extra_args: str, use_gpu: bool, name: str, env=()):
    """The example task, as ``dstack apply`` would submit it, run from this checkout."""
    import yaml

    from dstack_amd.core.models.configurations import parse_run_configuration

    with open(EXAMPLE) as f:
        conf = yaml.safe_load(f)
    cmds = list(conf["commands"])
    train = re.sub(r"--steps \d+", f"--steps {steps}", cmds[-1])
    train = re.sub(r"--warmup \d+", f"--warmup {warmup}", train)
    conf["commands"] = [f"cd {REPO}", *cmds[:-1], train + (" " + extra_args if extra_args else "")]
    conf["name"] = name
    conf.pop("image", None)  # process driver: the host's environment is the job's environment
    if use_gpu:
        conf["resources"] = {"gpu": f"MI355X:{gpus}"}
    else:
        conf["resources"] = {"cpu": "1..", "gpu": 0}
    # a rendezvous port of its own: under the driver's torchrun (bench.py --gpus N) the default
    # 29500 may be the outer job's store, and the RCCL pre-flight takes the next port too
    conf["env"] = list(conf.get("env", [])) + [f"PYTHONPATH={REPO}", "OMP_NUM_THREADS=1",
                                               f"MASTER_PORT={_free_port_pair()}"]
    if env:  # --env overrides (e.g. DSTACK_RCCL_PREFLIGHT=force|0 for the pre-flight A/B); the last wins
        last = {e.split("=", 1)[0]: e for e in env}
        conf["env"] = [e for e in conf["env"] if e.split("=", 1)[0] not in last] + list(last.values())
    return parse_run_configuration(conf)


def _parse_logs(text: str):
    stages, result = None, None
    for line in text.splitlines():
        if line.startswith("[train] stages "):
            try:
                stages = json.loads(line[len("[train] stages "):])
            except ValueError:
                pass
        elif line.startswith("{") and '"metric"' in line:
            try:
                result = json.loads(line)
            except ValueError:
                pass
    return stages, result


def one_run(client, conf, timeout: float) -> dict:
    t0 = time.time()
    run = client.runs.submit(conf)
    run.wait(timeout=timeout, poll=0.1)
    logs = b"".join(run.logs()).decode(errors="replace")
    sub = run.model.jobs[0].job_submissions[-1]
    timings = dict(sub.timings or {})
    timings.setdefault("submitted", t0)
    stages, result = _parse_logs(logs)
    stamps = dict(timings)
    if stages:
        stamps.update({k: v for k, v in stages.items() if isinstance(v, (int, float))})
    out = {"status": sub.status.value, "instance": sub.job_provisioning_data.instance_id if sub.job_provisioning_data else None,
           "stages_s": {}, "job_result": result}
    for name, a, b in STAGES:
        if a in stamps and b in stamps:
            out["stages_s"][name] = round(stamps[b] - stamps[a], 4)
    if "first_step_done" in stamps:
        out["time_to_first_step_s"] = round(stamps["first_step_done"] - stamps["submitted"], 4)
        out["time_to_train_start_s"] = round(stamps["model_ready"] - stamps["submitted"], 4)
    if "first_log" in timings:
        out["time_to_first_log_s"] = round(timings["first_log"] - timings["submitted"], 4)
    if stages and stages.get("first_step_split"):
        out["first_step_split"] = stages["first_step_split"]
    pf = next((ln for ln in logs.splitlines() if ln.startswith("[dstack] RCCL pre-flight")), None)
    if pf:  # the runner's own line: mode, duration and exit of the probe
        out["preflight"] = pf[:200]
    if stages is None or (result is None and out["status"] != "done"):
        out["log_tail"] = logs[-2000:]
    return out


def measure(gpus: int = 1, runs: int = 3, steps: int = 1, warmup: int = 1, tok_steps: int = 5, tok_warmup: int = 2,
            extra_args: str = "", timeout: float = 600.0, gpu: str = "auto", fake_gpus: int = 0, env=(),
            local_probe: bool = False) -> dict:
    """``fake_gpus`` > 0 (CPU tests): the agents see that many MI355X in a fake sysfs/KFD tree and
    the task's ranks run on the CPU over gloo."""
    for k in _LAUNCHER_ENV:
        os.environ.pop(k, None)
    from bench_coldstart import _host_has_gpu, _retire_instances
    from dstack_amd.server.testing import ServerProcess

    srv_env = {"DSTACK_LOCAL_SHIM_PER_INSTANCE": "1"}
    if local_probe:  # the shim hands dstack-probe to the runner (the example's RCCL pre-flight runs)
        srv_env["DSTACK_LOCAL_GPU_PROBE"] = "1"
    if fake_gpus:
        import tempfile

        from dstack_amd.server.testing import fake_amd_sysfs

        srv_env["DSTACK_SYSFS_ROOT"] = fake_amd_sysfs(tempfile.mkdtemp(prefix="dsa_sysfs_"), n_gpus=fake_gpus)
        use_gpu = True
    else:
        use_gpu = _host_has_gpu() if gpu == "auto" else gpu == "yes"
    samples, errors = [], []
    with ServerProcess(env=srv_env) as srv:
        client = srv.client()
        for i in range(runs + (1 if tok_steps else 0)):
            if i > 0 and not _retire_instances(client):
                errors.append(f"run {i}: previous instance still active")
            tok_run = i == runs
            conf = task_conf(gpus, tok_steps if tok_run else steps, tok_warmup if tok_run else warmup, extra_args,
                             use_gpu, f"llama3-apply-{i}", env)
            s = one_run(client, conf, timeout)
            s["kind"] = "tokens" if tok_run else "cold"
            samples.append(s)
            if s["status"] != "done" or "time_to_first_step_s" not in s:
                errors.append(f"run {i}: {s.get('status')}: {s.get('log_tail', '')[-400:]}")
    cold = [s for s in samples if s["kind"] == "cold" and "time_to_first_step_s" in s]
    p50 = (lambda xs: round(statistics.median(xs), 4) if xs else None)
    stage_p50 = {name: p50([s["stages_s"][name] for s in cold if name in s["stages_s"]]) for name, _, _ in STAGES}
    tok = next((s for s in samples if s["kind"] == "tokens"), None)
    job_res = (tok or {}).get("job_result") or {}
    return {
        "time_to_first_step_p50_s": p50([s["time_to_first_step_s"] for s in cold]),
        "time_to_train_start_p50_s": p50([s["time_to_train_start_s"] for s in cold]),
        "time_to_first_log_p50_s": p50([s["time_to_first_log_s"] for s in cold if "time_to_first_log_s" in s]),
        "stages_p50_s": stage_p50,
        "runs": len(cold), "distinct_instances": len({s["instance"] for s in samples if s["instance"]}),
        "gpus": gpus, "gpu_requested": f"MI355X:{gpus}" if use_gpu else None,
        "job_tokens_per_s": job_res.get("value"), "job_ms_per_step": job_res.get("ms_per_step"),
        "job_steps": job_res.get("steps"), "job_n_gpus": job_res.get("n_gpus"),
        "excludes": "VM boot, image pull, container start (local backend, process driver)",
        "errors": errors[:5], "samples": samples,
    }


def _interleaved(a) -> int:
    """Same-box A/B of task env switches: ``--runs`` rounds, each arm once per round (a fresh
    server and instance per measurement), p50 of time-to-first-step and of its stages per arm."""
    arms = [x.strip() for x in a.interleave.split(",") if x.strip()]
    per = {arm: [] for arm in arms}
    for _ in range(a.runs):
        for arm in arms:
            r = measure(a.gpus, 1, a.steps, a.warmup, 0, 0, a.extra_args, a.timeout, a.gpu, a.fake_gpus,
                        [*a.env, arm], a.local_probe)
            per[arm].append({"first_step_s": r["stages_p50_s"].get("first_step_s"), "stages_s": r["stages_p50_s"],
                             "time_to_first_step_s": r["time_to_first_step_p50_s"], "errors": r["errors"],
                             "preflight": next((x.get("preflight") for x in r["samples"] if x.get("preflight")),
                                               None),
                             "first_step_split": next((x.get("first_step_split") for x in r["samples"]
                                                       if x.get("first_step_split")), None)})
    p50 = (lambda xs: round(statistics.median(xs), 4) if xs else None)
    out = {arm: {"first_step_p50_s": p50([x["first_step_s"] for x in v if x["first_step_s"] is not None]),
                 "time_to_first_step_p50_s": p50([x["time_to_first_step_s"] for x in v
                                                  if x["time_to_first_step_s"] is not None]),
                 "samples": v} for arm, v in per.items()}
    print(json.dumps(out), flush=True)
    return 0 if all(not x["errors"] for v in per.values() for x in v) else 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--runs", type=int, default=3, help="fresh-instance runs for the time-to-first-step p50")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--tok-steps", type=int, default=5, help="timed steps of the final tokens/s run (0: none)")
    ap.add_argument("--tok-warmup", type=int, default=2)
    ap.add_argument("--extra-args", default="", help="appended to the task's bench.py command (e.g. a small model)")
    ap.add_argument("--timeout", type=float, default=600)
    ap.add_argument("--gpu", choices=("auto", "yes", "no"), default="auto")
    ap.add_argument("--fake-gpus", type=int, default=0, help="CPU tests: agents see N fake MI355X (gloo ranks)")
    ap.add_argument("--env", action="append", default=[], help="KEY=VALUE for the task's env (repeatable)")
    ap.add_argument("--local-probe", action="store_true", help="hand dstack-probe to the runner (pre-flight runs)")
    ap.add_argument("--interleave", default="", help="A/B: comma-separated env assignments, one arm each; the "
                                                     "runs alternate between the arms")
    a = ap.parse_args()
    if a.interleave:
        return _interleaved(a)
    r = measure(a.gpus, a.runs, a.steps, a.warmup, a.tok_steps, a.tok_warmup, a.extra_args, a.timeout, a.gpu,
                a.fake_gpus, a.env, a.local_probe)
    print(json.dumps(r), flush=True)
    return 0 if not r["errors"] else 1


if __name__ == "__main__":
    sys.exit(main())
