#!/usr/bin/env python3
"""Host cost of bench.py's per-frame band exchange on one GPU: torch.distributed over RCCL with world size 1, the
rank sending to and receiving from itself (RCCL allows a self peer inside a group), k send/receive pairs per
frame as the display rank of an N = k + 1 gather posts, through the same calls bench.py's gather_bands makes
(P2POp, batch_isend_irecv, stream wait). Prints the host microseconds per frame and the frames/s the exchange
alone sustains; the GPU work per frame is the copies only (no render)."""
import os
import sys
import time

import torch
import torch.distributed as dist


def main(k=7, nbytes=1_600_000, frames=2000):
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    src = [torch.empty(nbytes, dtype=torch.uint8, device=dev) for _ in range(k)]
    dst = [torch.empty(nbytes, dtype=torch.uint8, device=dev) for _ in range(k)]
    st = torch.cuda.Stream(dev)
    for it in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        host = 0.0
        with torch.cuda.stream(st):
            for _ in range(frames):
                h0 = time.perf_counter()
                ops = []
                for s, d in zip(src, dst):
                    ops.append(dist.P2POp(dist.isend, s, 0))
                    ops.append(dist.P2POp(dist.irecv, d, 0))
                works = dist.batch_isend_irecv(ops)
                for w in works:
                    w.wait()
                host += time.perf_counter() - h0
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"k={k} pairs of {nbytes} B: host {host / frames * 1e6:.1f} us per frame, wall {dt / frames * 1e6:.1f} us "
              f"per frame ({frames / dt:.0f} frames/s)", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main(*(int(x) for x in sys.argv[1:]))
