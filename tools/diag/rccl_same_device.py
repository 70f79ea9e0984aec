"""Can two RCCL ranks share one GPU?  Two processes, both on cuda:0, init_process_group("nccl") and run
one all-reduce, reduce-scatter and all-gather; prints what happened per rank.  (NCCL refuses a
duplicate device at communicator init; this checks what RCCL does on this box.)"""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    try:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
        x = torch.full((1 << 20,), float(rank + 1), device="cuda")
        dist.all_reduce(x)
        out = torch.empty(1 << 19, device="cuda")
        dist.reduce_scatter_tensor(out, torch.ones(1 << 20, device="cuda"))
        full = torch.empty(1 << 20, device="cuda")
        dist.all_gather_into_tensor(full, out)
        torch.cuda.synchronize()
        print(f"rank {rank}: ok all_reduce={x[0].item()} reduce_scatter={out[0].item()} all_gather={full[-1].item()}",
              flush=True)
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 -- report and exit non-zero
        print(f"rank {rank}: {type(e).__name__}: {e}", flush=True)
        sys.exit(3)


if __name__ == "__main__":
    mp.start_processes(worker, args=(2, 29611), nprocs=2, start_method="spawn")
