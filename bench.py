#!/usr/bin/env python3
"""Headline benchmark: tokens/sec of the Llama-3-8B training task (BASELINE.json metric).

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 it is launched under
``torch.distributed.run`` with one rank per GPU (RCCL over xGMI).  Started for N>1 WITHOUT a
launcher (no ``WORLD_SIZE``), it starts ``torch.distributed.run`` itself as a child process; a
``WORLD_SIZE`` that differs from ``--gpus`` is an error (exit 2), never a silently smaller run.  W untimed warmup steps, then
exactly K timed steps bracketed by barrier + ``torch.cuda.synchronize()``; the elapsed time is the
MAX over ranks; rank 0 prints one JSON line.  Every timed step is a full training step: forward,
backward, ZeRO-1 reduce-scatter, fused AdamW, all-gather.

Weak scaling: each GPU processes ``--grad-accum`` × ``--micro-batch`` × ``--seq-len`` tokens per
step (default 8 × 1 × 8192).
Data: synthetic random token ids; weights: random init (no network, no checkpoints).

The orchestration half of the metric is measured literally, in a child process with its own time
limit (``bench_apply.py``), at a moment when no rank of this benchmark holds a GPU:

* no launcher (N=1, or N>1 self-launched): in THIS process before any rank exists -- nothing here
  has touched the GPU yet, and the ranks are started only after the cold start has finished;
* under an external launcher (the driver's ``torch.distributed.run``): on rank 0 AFTER the timed
  steps, once every rank has freed its model, optimizer and cached blocks and left the process
  group (ranks 1..N-1 exit; rank 0 keeps only its idle HIP context), so the applied N-GPU task
  never shares HBM or xGMI links with the benchmark's own ranks and no collective waits on it.

In it a real server (native shim/runner, local backend) receives ``examples/llama3-8b-train`` through the API with ``MI355X:N``, the
task's own ``torchrun ... bench.py`` runs, and
``cold_start_p50_s`` = submit -> the task's FIRST OPTIMIZER STEP finished, p50 over 3 runs that
each land on a freshly created instance (``cold_start.stages_p50_s`` splits it: control plane,
launch, imports, rendezvous, extension load, GEMM selections, model init, first step);
``job_tokens_per_s`` is the tokens/s that task printed itself.  ``cold_start.control_plane`` keeps
the control-plane-only number (submit -> first output of ``echo ready``, ``bench_coldstart.py``).
Not included (local backend): VM boot, image pull, container start.  ``--no-coldstart`` skips it.
"""

from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

METRIC = "p50 job cold-start (s) + tokens/sec of 8-GPU Llama-3-8B task via dstack apply"
BASELINE_VALUE = None  # BASELINE.json "published": {} — the reference publishes no number


def _child_json(cmd: list, timeout: float) -> dict:
    """Run a measurement script as a child process (this process has not touched the GPU) and
    return its last JSON line."""
    import subprocess

    here = os.path.dirname(os.path.abspath(__file__))
    try:
        r = subprocess.run([sys.executable, *cmd], capture_output=True, text=True, timeout=timeout, cwd=here)
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        if lines:
            return json.loads(lines[-1])
        return {"error": (r.stderr or r.stdout)[-300:]}
    except (subprocess.TimeoutExpired, OSError, ValueError) as e:
        return {"error": str(e)[:300]}


def _cold_start(args) -> dict:
    """The task through ``dstack apply`` (bench_apply.py) and the control-plane-only cold start
    (bench_coldstart.py).  ``--coldstart-fake-gpus`` (CPU tests): the agents see that many fake
    MI355X and the task's ranks run on the CPU over gloo."""
    model_args = (f"--model {args.model} --seq-len {args.seq_len} --micro-batch {args.micro_batch} "
                  f"--grad-accum {args.grad_accum}")
    cmd = ["bench_apply.py", "--gpus", str(args.gpus), "--runs", "3", "--steps", "1", "--warmup", "1",
           "--tok-steps", "5", "--tok-warmup", "2", "--extra-args", model_args,
           "--timeout", str(args.coldstart_timeout)]
    if args.coldstart_fake_gpus:
        cmd += ["--fake-gpus", str(args.coldstart_fake_gpus)]
    # 4 task runs, each bounded by --timeout inside; the child as a whole by 4x that
    apply = _child_json(cmd, 4 * args.coldstart_timeout + 120)
    apply.pop("samples", None)
    cp = _child_json(["bench_coldstart.py", "--runs", "5", "--warm-runs", "4"], 180.0)
    apply["control_plane"] = {k: cp.get(k) for k in ("cold_start_p50_s", "stages_p50_s", "warm_start_p50_s",
                                                      "fresh_ok", "fresh_runs", "error") if cp.get(k) is not None}
    return apply


def _merge_cold(out: dict, cold: dict | None) -> dict:
    """Submit -> first optimizer step of the example task applied through the server, p50 over
    fresh instances, and the task's own tokens/s, next to the in-process number."""
    if cold is None:
        return out
    out["cold_start_p50_s"] = cold.get("time_to_first_step_p50_s")
    out["job_tokens_per_s"] = cold.get("job_tokens_per_s")
    out["cold_start"] = {k: cold.get(k) for k in ("time_to_train_start_p50_s", "time_to_first_log_p50_s",
                                                  "stages_p50_s", "runs", "distinct_instances",
                                                  "gpu_requested", "job_ms_per_step", "job_steps",
                                                  "job_n_gpus", "excludes", "errors", "error",
                                                  "control_plane", "when")
                         if cold.get(k) not in (None, [])}
    return out


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _self_launch(n: int, argv: list, cold: dict | None) -> int:
    """``bench.py --gpus N`` (N>1) started without a launcher: run N ranks under
    ``torch.distributed.run`` as a CHILD process (nothing here has touched the GPU, and no exec
    replaces this process), forward its output, and return its exit code.  The cold start has
    already run in this process, before any rank existed; it is merged into rank 0's JSON line
    here.  That line must report ``n_gpus == N``; anything else is an error, never a silent 1-GPU
    number."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv,
           "--no-coldstart"]
    env = dict(os.environ, DSTACK_AMD_BENCH_CHILD="1")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    result = None
    for line in proc.stdout:
        if line.startswith("{"):
            try:
                result = json.loads(line)
                continue  # printed once, with the cold start merged in, after the ranks exit
            except ValueError:
                pass
        sys.stdout.write(line)
        sys.stdout.flush()
    rc = proc.wait()
    if rc != 0:
        return rc
    if result is None or result.get("n_gpus") != n:
        print(f"error: expected a result line with n_gpus={n}, got {result and result.get('n_gpus')}",
              file=sys.stderr)
        return 3
    print(json.dumps(_merge_cold(result, cold)), flush=True)
    return 0


def _release_gpu() -> None:
    """Every rank drops its model, optimizer and cached HBM blocks and leaves the process group
    (RCCL communicators included), so nothing of the benchmark competes with the cold-start task
    and no collective or watchdog waits while rank 0 measures it."""
    import gc

    import torch
    import torch.distributed as dist

    gc.collect()  # (the caller has closed and dropped its trainer)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        held = torch.cuda.memory_allocated() / 2**30
        if held > 1.0:  # the cold-start task needs the GPUs: say so if this rank could not let go
            print(f"[bench] warning: {held:.1f} GiB still allocated after releasing the trainer", file=sys.stderr,
                  flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--seq-len", type=int, default=8192)
    # 1 x 8192 tokens per micro-batch: 2 x 8192 (grad-accum 4, same tokens/step, 207 vs 171 GB)
    # measured 1.2 % slower, interleaved on one box (profiles/ab_microbatch_r4p.txt)
    ap.add_argument("--micro-batch", type=int, default=1)
    # 8 x 8192-token micro-batches per optimizer step: 64k tokens/GPU/step, a 0.5M-token global
    # batch at 8 GPUs (Llama-3 pre-training used 4M+).  It amortises the HBM-bound fp32 AdamW pass
    # (~36 ms/step on one GPU) and the ZeRO-1 collectives; same box, tokens/s: 2 -> 20.96k,
    # 4 -> 21.49k, 8 -> 21.81k (profiles/ab_r2l_grad_accum.txt)
    ap.add_argument("--grad-accum", type=int, default=8)
    ap.add_argument("--no-coldstart", action="store_true", help="skip the dstack-apply cold-start half")
    ap.add_argument("--coldstart-timeout", type=float, default=600.0, help="time limit of one applied task run")
    ap.add_argument("--coldstart-fake-gpus", type=int, default=0, help=argparse.SUPPRESS)  # CPU tests
    args = ap.parse_args()

    launched = "WORLD_SIZE" in os.environ
    cold = None
    if not launched:
        # no rank exists and nothing in this process has touched the GPU: the cold start runs now
        if not args.no_coldstart:
            cold = dict(_cold_start(args), when="before the benchmark's ranks started")
        if args.gpus > 1:
            sys.exit(_self_launch(args.gpus, sys.argv[1:], cold))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"error: --gpus {args.gpus} but WORLD_SIZE={world}: one rank per GPU is required", file=sys.stderr)
        sys.exit(2)

    from dstack_amd.workloads.train_llama import run

    env, tr, res = run(args.model, args.seq_len, args.micro_batch, args.steps, args.warmup, log_every=0,
                       grad_accum=args.grad_accum)
    if env.world != args.gpus:
        print(f"error: joined a group of {env.world} ranks, --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    import torch

    out = None
    if env.rank == 0:
        out = {
            "metric": METRIC,
            "value": round(res["tokens_per_s"], 2),
            "unit": "tokens/s",
            "n_gpus": env.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(res["ms_per_step"], 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (res["tokens_per_s"] / BASELINE_VALUE) if BASELINE_VALUE else None,
            "dtype": "bf16",
            "data": "synthetic (Zipf unigram + bigram chains, fresh batch every micro-step; "
                    "workloads/data.py), random-init weights",
            "config": {
                "model": "Llama-3-8B" if args.model == "llama-3-8b" else args.model,
                "global_batch": args.micro_batch * args.grad_accum * env.world,
                "micro_batch": args.micro_batch,
                "grad_accum": args.grad_accum,
                "seq_len": args.seq_len,
                "parallelism": f"dp{env.world}" + ("-zero1" if env.world > 1 else ""),
                "optimizer": "AdamW (fp32 master, fused HIP kernel)",
            },
            "tflops_per_gpu": round(res["tflops_per_gpu"], 1),
            "final_loss": res["final_loss"],
            "losses": {"warmup": res.get("warmup_losses"), "timed": res.get("losses"),
                       "floor": res.get("loss_floor"), "unigram_entropy": res.get("unigram_entropy")},
            "max_mem_gb": res["max_mem_gb"],
            "ops": os.environ.get("DSTACK_AMD_OPS", "hip"),
            "gemm_tuning": res.get("gemm_tuning"),
            "attn": os.environ.get("DSTACK_AMD_ATTN", "hip"),
            "device": torch.cuda.get_device_name(0) if torch.cuda.is_available() else "cpu",
        }
    tr.close()  # the optimizer's autograd hooks pin model and buffers from the C++ side
    del tr
    _release_gpu()
    if env.rank != 0:
        return
    if launched and not args.no_coldstart:
        # external launcher: the other ranks have left; the applied task gets the whole node
        cold = dict(_cold_start(args), when="after the timed steps; benchmark ranks released their GPUs")
    print(json.dumps(_merge_cold(out, cold)), flush=True)


if __name__ == "__main__":
    main()
