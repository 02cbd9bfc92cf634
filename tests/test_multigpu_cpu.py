"""N > 1 path on the CPU: world-size-2 (and 4) gloo process groups run bench.py's band partition,
band all-gather and max-over-ranks timing. Each rank renders its row band with the oracle (the
CPU stand-in for its GPU's k_raster band), and the gathered frame must equal a full-frame render.
Sort-first bands are exact: a pixel depends only on the triangles covering it.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, scene_name, out_dir, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "3d-renderer_amd", "python"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch
    import torch.distributed as dist

    import bench
    import oracle_py
    import scene_cases as sc

    dist.init_process_group("gloo", rank=rank, world_size=world)
    scene = getattr(sc, scene_name)()
    W, H = scene.width, scene.height
    y0, y1 = bench.band_rows(H, world, rank)
    col, dep, _ = oracle_py.render(scene, band=(y0, y1), threads=2)
    band = torch.from_numpy(np.ascontiguousarray(col).view(np.int32).reshape(-1).copy())
    dband = torch.from_numpy(np.ascontiguousarray(dep).view(np.int32).reshape(-1).copy())
    frame = torch.empty(H * W, dtype=torch.int32)
    dframe = torch.empty(H * W, dtype=torch.int32)
    out = bench.gather_bands(frame, band, world, mode=mode, rank=rank)
    dout = bench.gather_bands(dframe, dband, world, mode=mode, rank=rank)
    slowest = bench.max_over_ranks(float(rank + 1), torch.device("cpu"), True)
    if out is not None:  # gather mode: only the display rank (0) holds the frame
        np.save(os.path.join(out_dir, f"frame{rank}.npy"), out.numpy())
        np.save(os.path.join(out_dir, f"depth{rank}.npy"), dout.numpy())
    np.save(os.path.join(out_dir, f"slowest{rank}.npy"), np.array([slowest]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,scene_name,mode", [(2, "c1_cube", "gather"), (4, "textured_grid", "gather"),
                                                   (2, "textured_grid", "allgather")])
def test_row_band_assembly_equals_full_frame(world, scene_name, mode, oracle, tmp_path):
    import torch.multiprocessing as mp

    import scene_cases as sc

    port = _free_port()
    mp.start_processes(_worker, args=(world, port, scene_name, str(tmp_path), mode), nprocs=world, join=True,
                       start_method="spawn")
    scene = getattr(sc, scene_name)()
    col, dep, _ = oracle.render(scene, threads=4)
    full = np.ascontiguousarray(col).view(np.int32).reshape(-1)
    dfull = np.ascontiguousarray(dep).view(np.int32).reshape(-1)
    for r in range(world):
        if mode == "allgather" or r == 0:
            assert np.array_equal(np.load(tmp_path / f"frame{r}.npy"), full), f"rank {r} colour"
            assert np.array_equal(np.load(tmp_path / f"depth{r}.npy"), dfull), f"rank {r} depth"
        else:
            assert not (tmp_path / f"frame{r}.npy").exists()
        assert float(np.load(tmp_path / f"slowest{r}.npy")[0]) == float(world)


def _ring_worker(rank, world, port, out_dir, mode):
    """bench.GatherRing over gloo: 5 frames through the double buffer, each band stamped with
    (frame, rank); every assembled frame must hold exactly that frame's bands."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    import bench

    dist.init_process_group("gloo", rank=rank, world_size=world)
    rows, W = 3, 5
    ring = bench.GatherRing(world, rows * W, world * rows * W, lambda n: torch.zeros(n, dtype=torch.int32), mode=mode,
                            rank=rank)
    assembled = []
    for k in range(5):
        band = ring.acquire()
        band.fill_(1000 * k + rank)  # the "render" of frame k into this rank's band
        ring.publish()
        if k % 2 == 1:  # read back every other frame only after its gather completed
            ring.drain()
            assembled.append((k, ring.frame.clone().numpy()))
    ring.drain()
    assembled.append((4, ring.frame.clone().numpy()))
    for k, fr in assembled:
        if mode == "allgather" or rank == 0:
            np.save(os.path.join(out_dir, f"ring{rank}_{k}.npy"), fr)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["gather", "allgather"])
def test_gather_ring_double_buffer(mode):
    import torch.multiprocessing as mp

    import tempfile

    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_ring_worker, args=(world, _free_port(), d, mode), nprocs=world, join=True,
                           start_method="spawn")
        for r in (range(world) if mode == "allgather" else [0]):
            for k in (1, 3, 4):
                fr = np.load(os.path.join(d, f"ring{r}_{k}.npy")).reshape(world, -1)
                for src in range(world):
                    assert (fr[src] == 1000 * k + src).all(), (r, k, src)


def test_band_rows_partition():
    sys.path.insert(0, ROOT)
    import bench

    for H, N in [(2160, 1), (2160, 2), (2160, 4), (2160, 8), (1080, 8), (480, 2)]:
        bands = [bench.band_rows(H, N, r) for r in range(N)]
        assert bands[0][0] == 0 and bands[-1][1] == H
        assert all(bands[i][1] == bands[i + 1][0] for i in range(N - 1))
        assert len({b[1] - b[0] for b in bands}) == 1
    with pytest.raises(ValueError):
        bench.band_rows(1081, 2, 0)
