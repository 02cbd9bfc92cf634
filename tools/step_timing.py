#!/usr/bin/env python3
"""Diagnostics for the bench's short-run penalty: ms/step of the C3 timed loop at
20 and 200 steps, after different amounts of untimed warm-up, with the GPU idle or busy before t0.

Each trial: `warm_ms` of back-to-back frames (untimed), synchronize, then `steps` timed frames exactly
as bench.timed_run times them. Prints one JSON line per trial plus the host enqueue time per step."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "3d-renderer_amd", "python"))

import torch  # noqa: E402

import bench  # noqa: E402


def trial(br, steps, warm_ms, idle_ms=0.0):
    br.warm()
    t_end = time.perf_counter() + warm_ms * 1e-3
    n = 0
    while n < 5 or time.perf_counter() < t_end:
        br.step()
        n += 1
    br.drain()
    br.synchronize()
    torch.cuda.synchronize(br.dev)
    if idle_ms:
        time.sleep(idle_ms * 1e-3)
    host = []
    t0 = time.perf_counter()
    for _ in range(steps):
        h = time.perf_counter()
        br.step()
        host.append(time.perf_counter() - h)
    t_enq = time.perf_counter() - t0
    br.drain()
    torch.cuda.synchronize(br.dev)
    dt = time.perf_counter() - t0
    return {"steps": steps, "warm_ms": warm_ms, "warm_frames": n, "idle_ms": idle_ms,
            "ms_per_step": dt / steps * 1e3, "enqueue_ms_per_step": t_enq / steps * 1e3,
            "first_enqueue_ms": host[0] * 1e3, "max_enqueue_ms": max(host) * 1e3}


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    torch.cuda.set_device(0)
    scene = bench.build_scene(cfg)
    br = bench.BandRenderer(scene, 0, 1, 0, inflight=2)
    for rep in range(2):
        for warm_ms in (0.0, 50.0, 300.0):
            for steps in (20, 200):
                print(json.dumps(trial(br, steps, warm_ms)), flush=True)
    for idle in (1.0, 20.0, 200.0):
        print(json.dumps(trial(br, 20, 300.0, idle)), flush=True)
    br.close()


if __name__ == "__main__":
    main()
