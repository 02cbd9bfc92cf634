#!/usr/bin/env python3
"""Probe: can two processes share one GPU in an RCCL communicator (torch.distributed nccl, both ranks on cuda:0)?
Used to decide whether the N > 1 exchange can be exercised on a one-GPU box. Prints the outcome per rank."""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    try:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        t = torch.full((4,), float(rank + 1), device=dev)
        dist.all_reduce(t)
        x = torch.full((1 << 20,), rank, dtype=torch.uint8, device=dev)
        if rank == 0:
            dist.recv(x, 1)
        else:
            dist.send(x, 0)
        torch.cuda.synchronize()
        print(f"rank {rank}: all_reduce {t.tolist()}, p2p ok={bool((x == 1).all())}", flush=True)
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        print(f"rank {rank}: failed: {type(e).__name__}: {str(e)[:300]}", flush=True)


if __name__ == "__main__":
    mp.start_processes(worker, args=(2, 29561), nprocs=2, join=True, start_method="spawn")
