"""``bench.py`` driver contract on CPU: one JSON line from rank 0 with the BASELINE metric, for
N=1 and for N=2 ranks under ``torch.distributed.run`` (gloo, 127.0.0.1 rendezvous)."""

import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--model", "llama-tiny", "--seq-len", "64", "--steps", "2", "--warmup", "1", "--grad-accum", "2",
        "--no-coldstart"]
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _json_lines(out: str):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


def _env():
    return dict(os.environ, OMP_NUM_THREADS="2", PYTHONPATH=REPO)


def test_bench_single_process_json():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "1", *ARGS], cwd=REPO, env=_env(), capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    d = lines[0]
    assert KEYS <= set(d)
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["value"] > 0
    assert d["metric"].startswith("p50 job cold-start")
    assert d["config"]["global_batch"] == 2 and d["config"]["seq_len"] == 64


@pytest.mark.slow
def test_bench_two_ranks_gloo():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", "29533", "bench.py", "--gpus", "2", *ARGS]
    r = subprocess.run(cmd, cwd=REPO, env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # only rank 0 prints
    d = lines[0]
    assert d["n_gpus"] == 2
    assert d["config"]["parallelism"] == "dp2-zero1"
    assert d["config"]["global_batch"] == 4


@pytest.mark.slow
def test_bench_self_launches_ranks_without_a_launcher():
    """``bench.py --gpus 2`` with no torchrun around it starts the 2 ranks itself (child launcher,
    gloo on CPU) and reports n_gpus 2 -- never a silent 1-process number."""
    env = {k: v for k, v in _env().items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", *ARGS], cwd=REPO, env=env, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    assert lines[0]["n_gpus"] == 2 and lines[0]["config"]["parallelism"] == "dp2-zero1"


def test_bench_world_size_mismatch_is_an_error():
    env = dict(_env(), WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", *ARGS], cwd=REPO, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 2
    assert not _json_lines(r.stdout)
    assert "WORLD_SIZE=1" in r.stderr


def _cold_args():
    return [a for a in ARGS if a != "--no-coldstart"] + ["--coldstart-fake-gpus", "2", "--coldstart-timeout", "240"]


def _check_cold(d, n):
    assert d["n_gpus"] == n and d["config"]["parallelism"] == f"dp{n}-zero1"
    c = d["cold_start"]
    assert c["job_n_gpus"] == n and c["runs"] == 3 and c["gpu_requested"] == f"MI355X:{n}", c
    assert not c.get("errors"), c
    assert d["cold_start_p50_s"] > 0 and d["job_tokens_per_s"] > 0
    return c


def _skip_without_agents():
    from dstack_amd.native_bin import runner_path, shim_path

    if not (shim_path() and runner_path()):
        pytest.skip("native agents not built")
    from dstack_amd.ops.build import is_current

    if not is_current():
        pytest.skip("HIP extension not built for the current sources (the example's build step would compile)")


@pytest.mark.slow
def test_bench_self_launched_runs_cold_start_before_ranks_exist():
    """The driver's N>1 command without a launcher: the parent measures ``dstack apply`` of the
    example with ``MI355X:2`` (fake GPUs, gloo ranks) BEFORE it starts the benchmark's ranks, then
    merges that into rank 0's single JSON line."""
    _skip_without_agents()
    env = {k: v for k, v in _env().items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", *_cold_args()], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    assert _check_cold(lines[0], 2)["when"].startswith("before")


@pytest.mark.slow
def test_bench_under_launcher_runs_cold_start_after_ranks_release():
    """The driver's exact N>1 form (``torch.distributed.run ... bench.py --gpus 2``, no
    ``--no-coldstart``): rank 0 runs the cold start only after the timed steps, once both ranks
    have dropped the trainer and left the process group; rank 1 exits, one JSON line."""
    _skip_without_agents()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", "29537", "bench.py", "--gpus", "2", *_cold_args()]
    r = subprocess.run(cmd, cwd=REPO, env=_env(), capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    assert _check_cold(lines[0], 2)["when"].startswith("after")
