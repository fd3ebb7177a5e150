"""Probe: two ranks on the one GPU of the box over RCCL (backend "nccl"),
one all-reduce.  Run as:
    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 tools/rccl_world2_probe.py
"""

from __future__ import annotations

import os

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ["RANK"])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
    x = torch.full((8,), float(rank + 1), device="cuda:0")
    dist.all_reduce(x)
    torch.cuda.synchronize()
    print(f"rank {rank}: {x[0].item()}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
