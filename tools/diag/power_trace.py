"""Power / clock trace of the training step: samples amdsmi (socket power, GFX clock, activity)
every 200 ms on a side thread while the Llama-3-8B bench step runs, to tell whether the step runs
at the power cap (clock below its maximum while the GPU is fully busy).

    python tools/diag/power_trace.py --steps 6
"""
import argparse
import json
import os
import statistics
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import amdsmi  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    amdsmi.amdsmi_init()
    handles = amdsmi.amdsmi_get_processor_handles()
    h = handles[0]
    samples, stop = [], threading.Event()

    def sample():
        while not stop.is_set():
            s = {"t": time.time()}
            try:
                p = amdsmi.amdsmi_get_power_info(h)
                s["power_w"] = p.get("current_socket_power") or p.get("average_socket_power")
            except Exception as e:  # noqa: BLE001
                s["power_err"] = str(e)[:80]
            try:
                c = amdsmi.amdsmi_get_clock_info(h, amdsmi.AmdSmiClkType.GFX)
                s["gfx_mhz"], s["gfx_max_mhz"] = c.get("clk"), c.get("max_clk")
            except Exception as e:  # noqa: BLE001
                s["clk_err"] = str(e)[:80]
            try:
                s["gfx_activity"] = amdsmi.amdsmi_get_gpu_activity(h).get("gfx_activity")
            except Exception:  # noqa: BLE001
                pass
            samples.append(s)
            time.sleep(0.2)

    from dstack_amd.workloads.train_llama import Trainer

    tr = Trainer("llama-3-8b", 8192, 1, torch.device("cuda", 0), grad_accum=8, lr_warmup=300)
    for _ in range(a.warmup):
        tr.step()
    torch.cuda.synchronize()
    th = threading.Thread(target=sample, daemon=True)
    th.start()
    t0 = time.time()
    for i in range(a.steps):
        tr.step()
        torch.cuda.synchronize()
        print(f"step {i + 1} t={time.time() - t0:.1f}s", flush=True)
    stop.set()
    th.join()
    busy = [s for s in samples if isinstance(s.get("power_w"), (int, float))]
    out = {"samples": len(samples), "step_s": (time.time() - t0) / a.steps}
    for k in ("power_w", "gfx_mhz", "gfx_activity"):
        v = [s[k] for s in busy if isinstance(s.get(k), (int, float))]
        if v:
            out[k] = {"mean": round(statistics.mean(v), 1), "min": min(v), "max": max(v)}
    out["gfx_max_mhz"] = next((s.get("gfx_max_mhz") for s in samples if s.get("gfx_max_mhz")), None)
    try:
        cap = amdsmi.amdsmi_get_power_cap_info(h)
        out["power_cap_w"] = cap.get("power_cap") / 1e6 if cap.get("power_cap", 0) > 1e5 else cap.get("power_cap")
    except Exception as e:  # noqa: BLE001
        out["power_cap_err"] = str(e)[:80]
    errs = {s.get("power_err") or s.get("clk_err") for s in samples} - {None}
    if errs:
        out["errors"] = sorted(errs)[:3]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
