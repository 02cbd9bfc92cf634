#!/usr/bin/env python3
"""Hot-path benchmark: frames/s of the HIP software rasterizer on BASELINE.json's configs.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c1]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

One step = one frame of Trident's graphics-pipeline stage: the per-frame UBO + draw-list update
(UpdateUniformBuffer / push constants, Renderer.cpp:5822-6051, :5110-5151) and the five gfx950
kernels (k_vertex, k_setup, k_clip, k_raster) over geometry resident in HBM. N > 1 = sort-first
row bands (geometry replicated) + an RCCL all-gather of the BGRA8 bands into the full frame on
every rank, double-buffered so frame k's gather overlaps frame k+1's kernels. value = whole frames
per second (strong scaling: a frame's work is fixed, N GPUs share it); latency_ms = one frame end
to end without overlap. Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "3d-renderer_amd", "python"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "frames/sec + Mpixels/sec at 1080p & 4K; achieved HBM GB/s vs roofline"


def build_scene(name):
    from trident_raster import scenes

    if name == "c3":
        return scenes.scene_c3_grid(3840, 2160, 708)
    if name == "c3trs":  # the C3 grid under a translate + yaw + uniform-scale ComposeTransform (general path)
        return scenes.scene_c3_trs(3840, 2160, 708)
    if name == "c2":
        return scenes.scene_c2_sphere(1920, 1080)
    if name == "c1":
        return scenes.scene_c1_cube(0, 640, 480)
    if name == "c5":
        return scenes.scene_c5_textured(3840, 2160, 708, 2048)
    raise SystemExit(f"unknown config {name}")


def band_rows(height, world, rank):
    """Rank's row band [y0, y1): equal contiguous bands (all_gather_into_tensor needs equal sizes)."""
    if height % world:
        raise ValueError(f"height {height} does not split into {world} equal row bands")
    rows = height // world
    return rank * rows, (rank + 1) * rows


def band_split(height, world, display_rows=None):
    """Every rank's row band [y0, y1), top to bottom. Default: equal bands (any remainder one row at a
    time). With display_rows, the display rank 0 takes that many rows and the others share the rest
    (sizes within one row): the display rank's band never crosses a link, so when the gather is the
    bottleneck a larger display band shortens every remote band's transfer (sort-first load balancing;
    autotune_split picks the size on the hardware). display_rows = 0: the display rank renders nothing and only
    assembles (receives and decodes the other N - 1 bands; the native exchange only). A list of N row counts gives
    every band's size (rebalance_split)."""
    if world == 1:
        return [(0, height)]
    if isinstance(display_rows, (list, tuple)):  # explicit per-rank row counts (rebalance_split)
        sizes = [int(n) for n in display_rows]
        if len(sizes) != world or sum(sizes) != height or sizes[0] < 0 or min(sizes[1:]) < 1:
            raise ValueError(f"band sizes {sizes} do not split {height} rows over {world} ranks")
    elif display_rows is None:
        base, rem = divmod(height, world)
        sizes = [base + (1 if r < rem else 0) for r in range(world)]
    else:
        d = int(display_rows)
        if d < 0 or height - d < world - 1:
            raise ValueError(f"display band of {d} rows leaves no rows for {world - 1} other ranks of {height}")
        base, rem = divmod(height - d, world - 1)
        sizes = [d] + [base + (1 if r < rem else 0) for r in range(world - 1)]
    bands, y = [], 0
    for n in sizes:
        bands.append((y, y + n))
        y += n
    return bands


class _Works:
    """The requests of one grouped send/recv as one handle (wait() = a stream wait on each)."""

    def __init__(self, works):
        self.works = works

    def wait(self):
        for w in self.works:
            w.wait()


DBP_SLOT_PIXELS, DBP_HEADER, DBP_MAX_SLOT = 4096, 160, 12448  # include/tri_raster.h TRI_DBP_*
_BITLEN = None


def _dbp_encode_np(px, slot):
    """The delta bit-plane format (band_codec.hip) in numpy, vectorised: the CPU (gloo) side of BandCodec. px: uint32[n]
    B8G8R8A8 words -> (uint8[nslots * slot] stream, largest slot's bytes)."""
    import numpy as np

    global _BITLEN
    if _BITLEN is None:
        _BITLEN = np.array([int(i).bit_length() for i in range(256)], np.uint32)
    n = px.size
    nslots = (n + DBP_SLOT_PIXELS - 1) // DBP_SLOT_PIXELS
    p = np.empty(nslots * DBP_SLOT_PIXELS, np.int64)
    p[:n] = px
    p[n:] = px[-1] if n else 0
    seg = p.reshape(nslots * 4, 1024)
    first = (seg[:, 0] & 0x00FFFFFF).astype(np.uint32)
    first[np.arange(nslots * 4) * 1024 >= n] = 0  # a segment past the band: empty
    prev = np.concatenate([seg[:, :1], seg[:, :-1]], axis=1)
    z = np.empty((nslots * 4, 1024, 3), np.uint32)
    for c in range(3):
        d = ((seg >> (8 * c)) - (prev >> (8 * c))) & 0xFF
        d = np.where(d >= 128, d - 256, d)
        z[..., c] = np.where(d >= 0, 2 * d, -2 * d - 1)
    z = z.reshape(nslots * 4, 16, 64, 3)
    widths = _BITLEN[z.max(axis=2)]  # [segments, 16, 3]
    lanes = np.arange(64, dtype=np.uint64)
    planes = np.stack([(((z >> j) & 1).astype(np.uint64) << lanes[None, None, :, None]).sum(axis=2, dtype=np.uint64)
                       for j in range(8)], axis=-1)  # [segments, 16, 3, 8]
    used = np.arange(8)[None, None, None, :] < widths[..., None]
    packed = (widths[..., 0] | (widths[..., 1] << 4) | (widths[..., 2] << 8)).astype(np.uint16)  # [segments, 16]
    out = np.zeros(nslots * slot, np.uint8)
    maxb = 0
    for sl in range(nslots):
        segs = slice(4 * sl, 4 * sl + 4)
        pay = planes[segs][used[segs]]
        hdr = np.zeros(DBP_HEADER // 4, np.uint32)
        hdr[0] = 8 * pay.size
        for w in range(4):
            hdr[4 + 9 * w] = first[4 * sl + w]
            hdr[4 + 9 * w + 1: 4 + 9 * w + 9] = packed[4 * sl + w].view(np.uint32)
        nb = DBP_HEADER + 8 * pay.size
        maxb = max(maxb, nb)
        o = out[sl * slot:(sl + 1) * slot]
        if nb > slot:
            o[:4] = hdr[:1].view(np.uint8)
            continue
        o[:DBP_HEADER] = hdr.view(np.uint8)
        o[DBP_HEADER:nb] = pay.view(np.uint8)
    return out, maxb


def _dbp_decode_np(stream, n, alpha, slot):
    """The inverse of _dbp_encode_np: uint32[n] with alpha restored (an overflowed slot's pixels stay 0)."""
    import numpy as np

    nslots = (n + DBP_SLOT_PIXELS - 1) // DBP_SLOT_PIXELS
    out = np.zeros(nslots * DBP_SLOT_PIXELS, np.uint32)
    lanes = np.arange(64, dtype=np.uint64)
    for sl in range(nslots):
        o = stream[sl * slot:(sl + 1) * slot]
        hdr = o[:DBP_HEADER].view(np.uint32)
        if DBP_HEADER + int(hdr[0]) > slot:
            continue
        pay = o[DBP_HEADER:DBP_HEADER + int(hdr[0])].view(np.uint64)
        k = 0
        for w in range(4):
            widths = hdr[4 + 9 * w + 1: 4 + 9 * w + 9].view(np.uint16).astype(np.int64)
            carry = int(hdr[4 + 9 * w])
            base = (4 * sl + w) * 1024
            for b in range(16):
                val = np.full(64, alpha << 24, np.int64)
                for c in range(3):
                    wc = (int(widths[b]) >> (4 * c)) & 15
                    zz = np.zeros(64, np.int64)
                    for j in range(wc):
                        zz |= ((pay[k] >> lanes) & np.uint64(1)).astype(np.int64) << j
                        k += 1
                    d = np.where(zz & 1, -((zz + 1) >> 1), zz >> 1)
                    val |= ((np.cumsum(d) + ((carry >> (8 * c)) & 0xFF)) & 0xFF) << (8 * c)
                out[base + 64 * b: base + 64 * b + 64] = val.astype(np.uint32)
                carry = int(val[63]) & 0x00FFFFFF
    return out[:n]


class BandCodec:
    """Lossless band transfer formats for a band whose alpha bytes all equal `alpha` (tri_frame_alpha
    proves it from the context's state):
      "bgr24": its B, G, R bytes (3 B per pixel; tri_pack_bgr24 / tri_unpack_bgr24);
      "dbp":   the delta bit-plane format (tri_dbp_pack / tri_dbp_unpack: per 64-pixel block and channel the bit planes
               of the zigzag-mapped pixel differences, in fixed slots of `slot_bytes` per 4096 pixels — C3's bands need
               about 1.6 B per pixel). Every rank uses the same slot size, agreed before the timed region
               (agree_slot), so each band's message size is known to both sides.
    On the GPU the HIP kernels run on torch's current stream; on the CPU (gloo tests) the same formats run in torch /
    numpy. The sender's flags: an alpha byte that differs (1), a slot that overflowed (2, "dbp" only); check() raises on
    either (the transfer was lossy)."""

    def __init__(self, alpha, device, mode="bgr24", slot_bytes=DBP_MAX_SLOT):
        import torch

        self.alpha = int(alpha)
        self.mode = mode
        self.slot = int(slot_bytes)
        self.flag = torch.zeros(2, dtype=torch.int32, device=device)
        self.gpu = device.type == "cuda"

    def bytes_for(self, n):
        """The message size of an n-pixel band."""
        if self.mode == "dbp":
            return (n + DBP_SLOT_PIXELS - 1) // DBP_SLOT_PIXELS * self.slot
        return 3 * n

    def max_slot_bytes(self, band):
        """dbp: the largest slot this band needs (packed once into a scratch stream at the format's maximum slot)."""
        import numpy as np
        import torch

        n = band.numel()
        if n == 0:  # an assemble-only display rank sends nothing
            return 0
        if not self.gpu:
            return _dbp_encode_np(band.numpy().view(np.uint32), DBP_MAX_SLOT)[1]
        from trident_raster import raster

        scratch = torch.empty((n + DBP_SLOT_PIXELS - 1) // DBP_SLOT_PIXELS * DBP_MAX_SLOT, dtype=torch.uint8,
                              device=band.device)
        fl = torch.zeros(2, dtype=torch.int32, device=band.device)
        raster.dbp_pack(band.data_ptr(), n, self.alpha, scratch.data_ptr(), DBP_MAX_SLOT, fl.data_ptr(),
                        torch.cuda.current_stream().cuda_stream)
        return int(fl[1].item())

    def pack(self, band, out):
        """band: int32[n] (B8G8R8A8) -> out: uint8[bytes_for(n)]."""
        import numpy as np
        import torch

        n = band.numel()
        if self.gpu:
            from trident_raster import raster

            cs = torch.cuda.current_stream().cuda_stream
            if self.mode == "dbp":
                raster.dbp_pack(band.data_ptr(), n, self.alpha, out.data_ptr(), self.slot, self.flag.data_ptr(), cs)
            else:
                raster.pack_bgr24(band.data_ptr(), out.data_ptr(), n, self.alpha, self.flag.data_ptr(), cs)
            return
        b = band.view(torch.uint8).view(n, 4)
        if bool((b[:, 3] != self.alpha).any()):
            self.flag[0] |= 1
        if self.mode == "dbp":
            st, maxb = _dbp_encode_np(band.numpy().view(np.uint32), self.slot)
            out.copy_(torch.from_numpy(st))
            if maxb > self.slot:
                self.flag[0] |= 2
            return
        out.view(n, 3).copy_(b[:, :3])

    def unpack(self, src, band):
        """src: uint8[bytes_for(n)] -> band: int32[n] with alpha restored."""
        import numpy as np
        import torch

        n = band.numel()
        if self.gpu:
            from trident_raster import raster

            cs = torch.cuda.current_stream().cuda_stream
            if self.mode == "dbp":
                raster.dbp_unpack(src.data_ptr(), n, self.alpha, self.slot, band.data_ptr(), cs)
            else:
                raster.unpack_bgr24(src.data_ptr(), band.data_ptr(), n, self.alpha, cs)
            return
        if self.mode == "dbp":
            band.copy_(torch.from_numpy(_dbp_decode_np(src.numpy(), n, self.alpha, self.slot).view(np.int32)))
            return
        b = band.view(torch.uint8).view(n, 4)
        b[:, :3].copy_(src.view(n, 3))
        b[:, 3].fill_(self.alpha)

    def unpack_many(self, srcs, bands):
        """unpack of several bands; "dbp" on the GPU decodes them all in one launch (tri_dbp_unpack_bands)."""
        if self.gpu and self.mode == "dbp" and len(srcs) > 1:
            import torch
            from trident_raster import raster

            raster.dbp_unpack_bands([s.data_ptr() for s in srcs], [b.data_ptr() for b in bands],
                                    [b.numel() for b in bands], self.alpha, self.slot,
                                    torch.cuda.current_stream().cuda_stream)
            return
        for src, band in zip(srcs, bands):
            self.unpack(src, band)

    def check(self):
        f = int(self.flag[0].item())
        if f & 1:
            raise RuntimeError("a band's alpha was not the promised uniform value: the band transfer was lossy")
        if f & 2:
            raise RuntimeError(f"a band needed more than the agreed {self.slot}-B slots: the dbp transfer was lossy")


class _Unpacked:
    """Receive-side handle of a packed gather on the GPU: the unpack ran on the assembly stream behind the
    receives; wait() makes the current stream wait for it (no host block)."""

    def __init__(self, event):
        self.event = event

    def wait(self):
        import torch

        torch.cuda.current_stream().wait_event(self.event)


def gather_bands(frame, band, world, async_op=False, mode="gather", rank=0, dst=0, spans=None, codec=None,
                 stage=None, asm_stream=None):
    """Assemble the full frame from the per-rank BGRA8 bands; band r lands at elements
    [spans[r][0], spans[r][0] + spans[r][1]) of the frame (default: equal bands, r * n).
    mode "gather" (default): onto the display rank `dst` only, as one grouped point-to-point exchange
    (RCCL ncclSend/ncclRecv over xGMI: each rank sends its band once, the display rank receives N-1 bands
    over N-1 links at once; bands may differ in size). The display rank's own band is copied in unless it
    already is the frame's view (BandRenderer renders it in place). "allgather": onto every rank
    (all_gather_into_tensor, equal bands only: (N-1)/N of the frame into every GPU).
    Returns the work handle (None for world 1) with async_op, else the assembled frame (None on a
    non-display rank in gather mode). gloo backs the same calls in the CPU tests.
    codec (gather mode only): bands travel as 3 bytes per pixel through `stage` (the sender's uint8[3n]
    buffer; on the display rank a dict rank -> uint8 buffer per remote band), unpacked into the frame on
    `asm_stream` (GPU) once received."""
    if world == 1:
        return None if async_op else band
    import torch.distributed as dist

    if mode == "allgather":
        work = dist.all_gather_into_tensor(frame, band, async_op=async_op)
        return work if async_op else frame
    if spans is None:
        n = band.numel()
        spans = [(r * n, n) for r in range(world)]
    if rank == dst:
        own = frame.narrow(0, *spans[dst])
        if own.data_ptr() != band.data_ptr():
            own.copy_(band)
        if codec is None:
            ops = [dist.P2POp(dist.irecv, frame.narrow(0, *spans[r]), r) for r in range(world) if r != dst]
        else:
            ops = [dist.P2POp(dist.irecv, stage[r], r) for r in range(world) if r != dst]
    else:
        if codec is not None:
            codec.pack(band, stage)  # on the current (render) stream, before the send that waits on it
        ops = [dist.P2POp(dist.isend, band if codec is None else stage, dst)]
    work = _Works(dist.batch_isend_irecv(ops))
    if codec is not None and rank == dst:
        if frame.is_cuda:
            import torch

            asm = asm_stream or torch.cuda.current_stream()
            with torch.cuda.stream(asm):
                work.wait()  # the assembly stream waits for the receives
                remote = [r for r in range(world) if r != dst]
                codec.unpack_many([stage[r] for r in remote], [frame.narrow(0, *spans[r]) for r in remote])
                ev = torch.cuda.Event()
                ev.record(asm)
            work = _Unpacked(ev)
        else:
            work.wait()
            for r in range(world):
                if r != dst:
                    codec.unpack(stage[r], frame.narrow(0, *spans[r]))
            work = _Works([])  # complete (a gloo request is waited for once)
    if async_op:
        return work
    work.wait()
    return frame if rank == dst else None


def agree_dbp_slot(codec, band, dist_on, margin=1.02):
    """The "dbp" slot size every rank uses: the largest slot any rank's band needs (a max over ranks), with a margin
    for frame-to-frame variation, rounded up to 16 B and capped at the format's maximum (which never overflows).
    Every rank calls it at the same point (the max is a collective)."""
    need = max_over_ranks(float(codec.max_slot_bytes(band)), band.device, dist_on)
    codec.slot = int(min(DBP_MAX_SLOT, (int(need * margin) + 15) // 16 * 16))
    return codec.slot


def max_over_ranks(value, device, dist_on):
    """The job's time is the slowest rank's time."""
    if not dist_on:
        return value
    import torch
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


class GatherRing:
    """Double-buffered band assembly for N > 1: frame k's all-gather (on the collective's stream)
    overlaps frame k+1's kernels (on the render stream). Before frame k+2 reuses slot k % 2, the
    render stream waits for frame k's gather (work.wait() is a stream wait; the host does not
    block). Throughput is then max(render, gather) per frame instead of their sum."""

    def __init__(self, world, band_elems, frame_elems, make, mode="gather", rank=0, dst=0, nbuf=None, spans=None,
                 codec=None, make_bytes=None):
        self.world, self.mode, self.rank, self.dst, self.spans = world, mode, rank, dst, spans
        self.codec = codec if (world > 1 and mode == "gather") else None
        self.nbuf = nbuf if nbuf else (2 if world > 1 else 1)
        keeps_frame = world > 1 and (mode == "allgather" or rank == dst)
        if keeps_frame and mode == "gather":
            # the display rank renders its band straight into the frame (no copy, no transfer)
            self.frames = [make(frame_elems) for _ in range(self.nbuf)]
            off, n = spans[dst] if spans else (dst * band_elems, band_elems)
            self.bands = [f.narrow(0, off, n) for f in self.frames]
        else:
            self.bands = [make(band_elems) for _ in range(self.nbuf)]
            self.frames = [make(frame_elems) for _ in range(self.nbuf)] if keeps_frame else self.bands
        self.pending = [None] * self.nbuf
        self.k = 0
        self.stage, self.asm_stream = [None] * self.nbuf, None
        if self.codec is not None:  # 3-byte staging per slot: the sender's packed band, the receiver's per rank
            sp = spans or [(r * band_elems, band_elems) for r in range(world)]
            if rank == dst:
                self.stage = [{r: make_bytes(self.codec.bytes_for(sp[r][1])) for r in range(world) if r != dst}
                              for _ in range(self.nbuf)]
                if self.frames[0].is_cuda:
                    import torch

                    self.asm_stream = torch.cuda.Stream(self.frames[0].device)
            else:
                self.stage = [make_bytes(self.codec.bytes_for(sp[rank][1])) for _ in range(self.nbuf)]

    @property
    def inbound_bytes(self):
        """Bytes the display rank receives per frame (0 elsewhere)."""
        if self.world == 1 or self.rank != self.dst or self.mode != "gather":
            return 0
        sp = self.spans or [(r * self.bands[0].numel(), self.bands[0].numel()) for r in range(self.world)]
        nbytes = (lambda n: 4 * n) if self.codec is None else self.codec.bytes_for
        return sum(nbytes(sp[r][1]) for r in range(self.world) if r != self.dst)

    def acquire(self):
        """The band buffer frame k renders into (after frame k-2's gather released it)."""
        i = self.k % self.nbuf
        if self.pending[i] is not None:
            self.pending[i].wait()
            self.pending[i] = None
        return self.bands[i]

    def publish(self):
        """Start frame k's gather of the band returned by acquire()."""
        i = self.k % self.nbuf
        self.pending[i] = gather_bands(self.frames[i], self.bands[i], self.world, async_op=True, mode=self.mode,
                                       rank=self.rank, dst=self.dst, spans=self.spans, codec=self.codec,
                                       stage=self.stage[i], asm_stream=self.asm_stream)
        self.k += 1

    def drain(self):
        for i, w in enumerate(self.pending):
            if w is not None:
                w.wait()
                self.pending[i] = None

    def check(self):
        """Host check (synchronising): every packed band kept the promised alpha."""
        if self.codec is not None:
            self.codec.check()

    @property
    def frame(self):
        """The most recently assembled frame (complete after drain())."""
        return self.frames[(self.k - 1) % self.nbuf]


_XFER_COMMS = []
XFER_COMMS = 3  # one RCCL communicator per frame in flight (the most the bench uses), each used on one stream
XFER_TIMEOUT_MS = 60000  # tri_xfer_set_timeout: a wait that outlasts it aborts the communicators and raises


def xfer_comms(lib, world, rank, device_index, dev):
    """The process's RCCL communicators for tri_xfer (the native band exchange), created once: for each, rank 0 draws
    a unique id, torch.distributed broadcasts its 128 bytes, and every rank joins (collective). If a later
    communicator cannot be created on some rank (the outcome is agreed over ranks after each), the exchange runs on
    the ones made so far: tri_xfer fences a communicator that several frames in flight share.
    Destroyed at exit."""
    import atexit
    import ctypes as C

    import torch
    import torch.distributed as dist
    from trident_raster import raster

    if _XFER_COMMS:
        return _XFER_COMMS
    for k in range(XFER_COMMS):
        uid = (C.c_uint8 * 128)()
        if rank == 0:
            raster._check(lib.tri_xfer_unique_id(uid))
        t = torch.tensor(list(bytes(uid)), dtype=torch.uint8, device=dev)
        dist.broadcast(t, src=0)
        uid = (C.c_uint8 * 128)(*t.cpu().tolist())
        comm = C.c_void_p()
        rc = lib.tri_xfer_comm_create(uid, world, rank, device_index, C.byref(comm))
        failed = max_over_ranks(1.0 if rc else 0.0, dev, True)  # agreed first, so that every rank takes one branch
        if failed:
            if not rc:
                lib.tri_xfer_comm_destroy(comm)
            if k == 0:  # no communicator at all, on every rank: the caller's fallback (torch.distributed) takes over
                if rc:
                    raster._check(rc)  # this rank's own error
                raise RuntimeError("tri_xfer_comm_create failed on another rank")
            print(f"bench.py: WARNING: RCCL communicator {k + 1} of {XFER_COMMS} could not be created; the native "
                  f"exchange shares {k} communicator(s) across its frames in flight", file=sys.stderr, flush=True)
            break
        _XFER_COMMS.append(comm)
    atexit.register(lambda: [lib.tri_xfer_comm_destroy(c) for c in _XFER_COMMS])
    return _XFER_COMMS


def arm_watchdog(seconds, phase):
    """N > 1: a host-side deadline for one phase of the run. If the phase does not finish in time (a rank stuck in
    a collective's host call, where no device-side deadline reaches), dump every thread's stack and exit the process
    non-zero, so torchrun ends the job instead of leaving 8 GPUs waiting. Re-armed at each phase; 0 disarms."""
    import faulthandler

    faulthandler.cancel_dump_traceback_later()
    if seconds > 0:
        print(f"bench.py: phase '{phase}' (watchdog {seconds:.0f} s)", file=sys.stderr, flush=True)
        faulthandler.dump_traceback_later(seconds, exit=True)


class BandRenderer:
    """One rank's share of a frame: rows [y0, y1) rendered into torch-owned device buffers, assembled
    by a GatherRing. `inflight` contexts take frames in turn, each on its own stream with its own work
    buffers and one shared copy of the geometry (tri_geometry), so frame k+1's front end (vertex, set-up)
    runs while frame k rasterises — the reference also keeps several frames in flight
    (Renderer::DrawFrame waits on the fence of the frame in flight two frames back, Renderer.cpp:752-772)."""

    def __init__(self, scene, rank, world, device_index, band_world=None, assembly="gather", inflight=1,
                 display_rows=None, pack="auto", exchange="native"):
        import ctypes as C

        import torch
        from trident_raster import abi, raster, scenes

        H, W = scene.height, scene.width
        if assembly == "allgather" and not band_world:  # equal bands (the all-gather needs equal sizes)
            self.bands = [band_rows(H, world, r) for r in range(world)]
        else:  # band_world: one band of an N-way split rendered alone (diagnostics, no collective)
            self.bands = band_split(H, band_world or world, display_rows)
        self.band = self.bands[rank]
        rows = self.band[1] - self.band[0]
        self.scene, self.rank, self.world, self.rows = scene, rank, world, rows
        self.dev = torch.device("cuda", device_index)
        self.inflight = max(1, inflight)
        native = exchange == "native" and world > 1 and assembly == "gather" and self.dev.type == "cuda"
        if rows == 0 and not (native or world == 1):
            raise ValueError("an assemble-only display rank (a band of 0 rows) needs the native exchange")
        self.spans = spans = [(y0 * W, (y1 - y0) * W) for y0, y1 in self.bands] if world > 1 else None
        # an assemble-only display rank (0 rows) never renders in the frame loop: its contexts cover one row, for the
        # frame's state (the proven alpha, statistics)
        cband = self.band if rows else (0, 1)
        self.depth = [torch.empty((cband[1] - cband[0]) * W, dtype=torch.float32, device=self.dev)
                      for _ in range(self.inflight)]
        self.geometry = raster.TriGeometry(device_index)
        self.geometry.upload(scene.vertices, scene.indices, scene.meshes)
        # Each context renders on a dedicated torch stream (a non-zero handle) that is torch's current
        # stream while its frame is enqueued and published: the collective then waits on the stream
        # k_raster wrote the band on, and work.wait() in GatherRing.acquire orders that same stream behind
        # the gather that read the slot. (Torch's default stream is handle 0, which tri_set_stream takes
        # as "the context's own non-blocking stream" — unordered with the collective.)
        self.rs, self.streams = [], []
        for _ in range(self.inflight):
            r = raster.TriRaster(W, H, band=cband, device=device_index)
            st = torch.cuda.Stream(self.dev)
            r.set_stream(st.cuda_stream)
            scenes.load_scene(r, scene, geometry=self.geometry)
            self.rs.append(r)
            self.streams.append(st)
        self.r = self.rs[0]
        # a compact band format when every pixel's alpha is provably one value (every rank proves the same from the
        # same scene, so sender and receiver agree without a message): the delta bit-plane format by default ("auto"),
        # or the 3-byte one
        self.alpha = self.r.frame_alpha()
        mode = {"auto": "dbp", "dbp": "dbp", "bgr24": "bgr24"}.get(pack)
        self.codec = BandCodec(self.alpha, self.dev, mode) if (mode and self.alpha >= 0 and world > 1 and
                                                                 assembly == "gather") else None
        self._lib = raster.load_library()
        self._raster = raster
        self.pack = pack
        if self.codec is not None and self.codec.mode == "dbp":  # the slot size every rank's band fits (collective)
            agree_dbp_slot(self.codec, self.probe_band(), world > 1)
        if native:  # tri_xfer owns the exchange (below): the ring keeps one band buffer, no frames or staging
            self.ring = GatherRing(1, rows * W, rows * W, lambda n: torch.empty(n, dtype=torch.int32, device=self.dev))
        else:
            self.ring = GatherRing(world, rows * W, H * W, lambda n: torch.empty(n, dtype=torch.int32, device=self.dev),
                                   mode=assembly, rank=rank, nbuf=max(self.inflight, 2 if world > 1 else 1),
                                   spans=spans, codec=self.codec,
                                   make_bytes=lambda n: torch.empty(n, dtype=torch.uint8, device=self.dev))
        # the per-frame calls with their ctypes arguments built once (a frame at N = 8 is ~60 us of GPU
        # work, so Python-side marshalling per call would show up in the frame rate)
        self._ctxs = [r._ctx for r in self.rs]
        self._ubo = C.byref(scene.ubo)
        self._clear = C.byref((C.c_float * 4)(*scene.clear))
        self._draws, self._ndraws = abi.draws_array(scene.draws)
        self._band_ptrs = {b.data_ptr(): C.c_void_p(b.data_ptr()) for b in self.ring.bands}
        self._depth_ptrs = [C.c_void_p(d.data_ptr()) for d in self.depth]
        # N > 1 gather on the GPU: the exchange runs natively (tri_xfer: one library call per frame renders the band
        # and sends it, or receives and decodes every remote band, over an RCCL communicator of the library's own);
        # torch.distributed's point-to-point calls cost the host ~20 us each (tools/p2p_host_cost.py), which at
        # N = 8 would bind the display rank far below one GPU's frame rate. The GatherRing above stays the
        # exchange for --exchange torch, the all-gather and the gloo tests.
        self.xfer, self._kx, self.xfer_comms = None, 0, 0
        if native:
            self._attach_xfer(device_index)
        self.frames = 0
        self.sim_step = None  # --sim-codec: the band codec's per-frame work, on the frame's stream

    def _attach_xfer(self, device_index):
        import ctypes as C

        import torch
        from trident_raster import abi

        lib, W, H = self._lib, self.scene.width, self.scene.height
        comms = xfer_comms(lib, self.world, self.rank, device_index, self.dev)
        self.nbuf = self.inflight  # slot i belongs to context i: its frames render and transfer on one stream
        n = H * W if self.rank == 0 else self.rows * W
        self.xbufs = [torch.empty(n, dtype=torch.int32, device=self.dev) for _ in range(self.nbuf)]
        fmt = {None: abi.TRI_GROUP_FMT_BGRA32, "bgr24": abi.TRI_GROUP_FMT_BGR24, "dbp": abi.TRI_GROUP_FMT_DBP}[
            self.codec.mode if self.codec is not None else None]
        band_y = (C.c_uint32 * (self.world + 1))(*([y0 for y0, _ in self.bands] + [H]))
        cfg = abi.TriXferConfig(W, band_y, 0, fmt, self.codec.slot if fmt == abi.TRI_GROUP_FMT_DBP else 0,
                                max(self.alpha, 0) if self.codec is not None else 0, self.nbuf)
        x = C.c_void_p()
        carr = (C.c_void_p * len(comms))(*[c.value for c in comms])
        self._raster._check(lib.tri_xfer_create(carr, len(comms), C.byref(cfg), C.byref(x)))
        self.xfer = x
        self._raster._check(lib.tri_xfer_set_timeout(x, XFER_TIMEOUT_MS))
        self.xfer_comms = len(comms)
        for s, b in enumerate(self.xbufs):
            self._raster._check(lib.tri_xfer_bind_slot(x, s, C.c_void_p(b.data_ptr())))

    def _xframe(self, i, exchange=1, render=True):
        """One frame through tri_xfer on context i, into its slot i (render=False, or an assemble-only display rank:
        the exchange alone)."""
        slot = i % self.nbuf
        self._kx = slot
        render = render and self.rows > 0
        rc = self._lib.tri_xfer_frame(self.xfer, slot, self._ctxs[i] if render else None,
                                      self._depth_ptrs[i] if render else None, self._ubo if render else None,
                                      self._clear if render else None, self._draws if render else None,
                                      self._ndraws, exchange)
        if rc:
            self._raster._check(rc)

    def check(self):
        """Every packed band kept the promised alpha and fitted its dbp slots (synchronising); raises if not."""
        if self.xfer is not None:
            self._raster._check(self._lib.tri_xfer_synchronize(self.xfer))
        else:
            self.ring.check()

    def inbound_bytes(self):
        """Bytes the display rank receives per frame (0 elsewhere)."""
        if self.xfer is None:
            return self.ring.inbound_bytes
        import ctypes as C

        sent, recv = C.c_uint64(), C.c_uint64()
        self._raster._check(self._lib.tri_xfer_info(self.xfer, C.byref(sent), C.byref(recv), None))
        return recv.value

    def assembled_frame(self):
        """The display rank's most recently assembled frame (int32[H * W], device), after a device synchronisation."""
        if self.xfer is not None:
            return self.xbufs[self._kx]
        return self.ring.frame

    def probe_band(self):
        """One frame of this rank's band on context 0, into a scratch buffer (synchronised; no collective). An
        assemble-only display rank probes the first sender's band instead (a scratch context)."""
        import ctypes as C

        import numpy as np
        import torch
        from trident_raster import scenes

        if self.rows == 0:
            with self._raster.TriRaster(self.scene.width, self.scene.height, band=self.bands[1],
                                        device=self.dev.index) as r:
                scenes.load_scene(r, self.scene, geometry=self.geometry)
                r.render_frame()
                col, _ = r.readback(depth=False)
            return torch.from_numpy(np.ascontiguousarray(col).view(np.int32).reshape(-1)).to(self.dev)
        band = torch.empty(self.rows * self.scene.width, dtype=torch.int32, device=self.dev)
        r = self.rs[0]
        self._raster._check(self._lib.tri_bind_output(r._ctx, C.c_void_p(band.data_ptr()), C.c_void_p(self.depth[0].data_ptr())))
        r.render_frame()
        r.synchronize()
        return band

    def _frame(self, i):
        if self.xfer is not None:
            self._xframe(i)
            return
        lib, ctx = self._lib, self._ctxs[i]
        band = self.ring.acquire()
        if self.rows:  # (--sim-world's assemble-only display rank renders nothing)
            rc = (lib.tri_bind_output(ctx, self._band_ptrs[band.data_ptr()], self._depth_ptrs[i]) or
                  lib.tri_set_frame(ctx, self._ubo, self._clear) or   # per-frame uniform update
                  lib.tri_set_draws(ctx, self._draws, self._ndraws) or  # per-frame draw list (push constants)
                  lib.tri_render(ctx))
            if rc:
                self._raster._check(rc)
        if self.sim_step is not None:
            self.sim_step(band)
        self.ring.publish()

    def step(self, first_only=False):
        """One frame, on the next context in turn (first_only: always context 0, no overlap)."""
        i = 0 if first_only else self.frames % self.inflight
        self.frames += 1
        if self.xfer is not None or (self.world == 1 and self.inflight == 1 and self.sim_step is None):
            self._frame(i)  # no torch stream context needed (the native exchange orders its own streams)
            return
        import torch

        with torch.cuda.stream(self.streams[i]):
            self._frame(i)

    def warm(self):
        """One synchronous frame per context (sizes the internal queues; re-renders after TRI_E_OVERFLOW)."""
        for r in self.rs:
            r.render_frame()

    def synchronize(self):
        for r in self.rs:
            r.synchronize()

    def close(self):
        if self.xfer is not None:
            self._lib.tri_xfer_destroy(self.xfer)
            self.xfer = None
        for r in self.rs:
            r.close()
        self.geometry.close()

    def drain(self):
        if self.xfer is not None:  # stream-ordered already: the caller's device synchronisation waits for it
            return
        import torch

        with torch.cuda.stream(self.streams[0]):
            self.ring.drain()

    def _sync(self, check=False):
        """Device synchronisation; with the native exchange, first its bounded wait (TRI_E_TIMEOUT raises instead of
        hanging on a transfer whose peer never comes), and with check its status flags (a lossy band raises)."""
        import torch

        if self.xfer is not None:
            f = self._lib.tri_xfer_synchronize if check else self._lib.tri_xfer_wait
            self._raster._check(f(self.xfer))
        if self.dev.type == "cuda":
            torch.cuda.synchronize(self.dev)

    def render_only_ms(self, frames=100):
        """Diagnostics (N > 1 line): this rank's frames rendered back to back with no assembly, ms per frame."""
        import torch

        self.drain()
        self._sync()
        t0 = time.perf_counter()
        for k in range(frames):
            i = k % self.inflight
            if self.xfer is not None:
                self._xframe(i, exchange=0)
                continue
            if self.rows == 0:
                continue
            lib, ctx = self._lib, self._ctxs[i]
            band = self.ring.bands[k % len(self.ring.bands)]
            with torch.cuda.stream(self.streams[i]):
                rc = (lib.tri_bind_output(ctx, self._band_ptrs[band.data_ptr()], self._depth_ptrs[i]) or
                      lib.tri_set_frame(ctx, self._ubo, self._clear) or lib.tri_set_draws(ctx, self._draws, self._ndraws)
                      or lib.tri_render(ctx))
            if rc:
                self._raster._check(rc)
        self._sync()
        return (time.perf_counter() - t0) * 1e3 / frames

    def assembly_only_ms(self, frames=100):
        """Diagnostics (N > 1 line): the band assembly alone (pack, send/receive, unpack), frames back to back
        with no rendering, ms per frame. Every rank must call it (it runs the collectives)."""
        import torch

        self.drain()
        self._sync()
        t0 = time.perf_counter()
        if self.xfer is not None:
            for k in range(frames):
                self._xframe(k % self.inflight, exchange=1, render=False)
            self._sync()
            return (time.perf_counter() - t0) * 1e3 / frames
        with torch.cuda.stream(self.streams[0]):
            for _ in range(frames):
                self.ring.acquire()
                self.ring.publish()
            self.ring.drain()
        self._sync()
        return (time.perf_counter() - t0) * 1e3 / frames

    def attach_sim_codec(self, mode):
        """--sim-codec (one GPU, no collective): every frame also runs the band codec's work of its rank at N > 1, on
        the frame's stream — a sender packs its band; the display rank (sim rank 0) decodes every other band of the
        split (its own band repeated to each band's size and packed once) — so the frame rate includes the codec's
        cost and its overlap with the other frames in flight. The link transfer itself is not simulated."""
        import torch

        band = self.ring.bands[0]
        codec = BandCodec(max(self.alpha, 0), self.dev, mode)
        if mode == "dbp":
            agree_dbp_slot(codec, self.probe_band(), False)
        if self.rank != 0:
            stage = torch.empty(codec.bytes_for(band.numel()), dtype=torch.uint8, device=self.dev)
            self.sim_step = lambda b: codec.pack(b, stage)
        else:
            W = self.scene.width
            remote = [(y1 - y0) * W for y0, y1 in self.bands[1:]]
            own = self.probe_band()
            srcs, views, frame = [], [], torch.empty(sum(remote), dtype=torch.int32, device=self.dev)
            off = 0
            for n in remote:
                src = torch.empty(codec.bytes_for(n), dtype=torch.uint8, device=self.dev)
                codec.pack(own.repeat((n + own.numel() - 1) // own.numel())[:n].contiguous(), src)
                srcs.append(src)
                views.append(frame.narrow(0, off, n))
                off += n
            self._sync()
            self.sim_step = lambda b: codec.unpack_many(srcs, views)
        self.sim_codec = codec

    def codec_ms(self, bands_rows, frames=200):
        """Diagnostics (--sim-world): the band codec's cost on one GPU: packing this rank's band, and the display
        rank's unpack of every other band of the split (ms per frame each). The remote bands' streams are this
        band's pixels repeated to each band's size and packed (real image content, the agreed slot size)."""
        import torch

        W = self.scene.width
        band = self.ring.bands[0] if self.rows else self.probe_band()
        codec = self.codec
        if codec is None:  # one GPU: the format --pack names, its slot agreed on this band alone
            codec = BandCodec(max(self.alpha, 0), self.dev, "bgr24" if self.pack == "bgr24" else "dbp")
            if codec.mode == "dbp":
                agree_dbp_slot(codec, band, False)
        st = torch.empty(codec.bytes_for(band.numel()), dtype=torch.uint8, device=self.dev)
        self._sync()
        t0 = time.perf_counter()
        for _ in range(frames):
            codec.pack(band, st)
        self._sync()
        pack = (time.perf_counter() - t0) * 1e3 / frames
        remote = [r * W for r in bands_rows[1:]]
        frame = torch.empty(sum(remote) + 16, dtype=torch.int32, device=self.dev)
        srcs = []
        for n in remote:
            src = torch.empty(codec.bytes_for(n), dtype=torch.uint8, device=self.dev)
            codec.pack(band.repeat((n + band.numel() - 1) // band.numel())[:n].contiguous(), src)
            srcs.append(src)
        views, off = [], 0
        for n in remote:
            views.append(frame.narrow(0, off, n))
            off += n
        self._sync()
        t0 = time.perf_counter()
        for _ in range(frames):
            codec.unpack_many(srcs, views)
        self._sync()
        unpack = (time.perf_counter() - t0) * 1e3 / frames
        return {"format": codec.mode, "slot_bytes": codec.slot if codec.mode == "dbp" else None,
                "pack_ms_per_band": pack, "unpack_ms_display_all_remote_bands": unpack,
                "remote_bands": len(remote), "band_pixels": band.numel(),
                "bytes_per_pixel": codec.bytes_for(band.numel()) / band.numel()}

    def latency_ms(self, frames=20):
        """Per-frame latency without overlap: render + gather + wait, host-synchronised each frame."""
        import torch

        self.drain()
        ts = []
        for _ in range(frames):
            self._sync()
            t0 = time.perf_counter()
            self.step()
            self.drain()
            self._sync()
            ts.append((time.perf_counter() - t0) * 1e3)
        ts.sort()
        return ts[len(ts) // 2]


# Frames in flight per config at N = 1 (round 4, same-box A/B of the whole bench line): the 1M-triangle 4K frame
# hides more of its front end behind the other frames' raster at 3 (C3 +2.3 %), while C2 and C5 lose 9-11 % at 3
# (their per-context buffers and the extra stream cost more than the overlap gains).
DEFAULT_INFLIGHT = {"c3": 3, "c3trs": 3, "c2": 2, "c5": 2, "c1": 2}


def split_candidates(height, world, min_rows=32, inflights=(2,), assemble_only=False):
    """(display rows, frames in flight) pairs autotune_split tries: the equal split, display bands up to 2.5x
    it (when the links bind, a larger display band shortens every remote band) and down to a quarter of it (when the
    display GPU's decode of the remote bands binds: a pixel moved off the display band costs it a decode, ~2 us per
    million pixels, instead of a render, ~20), as long as every band keeps at least `min_rows` rows (one bin
    row), at each frame count in `inflights` (a band's kernels are short at large N, and a third frame in flight
    keeps more of the GPU busy: N = 8 rank 4 on one GPU 33.4k frames/s with 2, 39.0k with 3, 33.1k with 4).
    assemble_only (the native exchange): also a display band of 0 rows — the display GPU renders nothing and only
    receives and decodes the other N - 1 bands, so it pays no front end of its own (a band's vertex and set-up
    kernels cost about as much at 67 rows as at 270)."""
    base = height / world
    ds = [int(round(base))]  # the equal split always (a small frame or a large world may leave no other)
    for m in (0.25, 0.5, 0.75, 1.25, 1.5, 2.0, 2.5):
        d = int(round(base * m))
        if d >= min_rows and height - d >= (world - 1) * min_rows and d not in ds:
            ds.append(d)
    if assemble_only and world > 2 and height >= (world - 1) * min_rows:
        ds.append(0)
    return [(d, k) for k in inflights for d in ds]


def measure_fps(br, frames, dist_on):
    """Whole-job frames/s of `frames` back-to-back frames (render + gather), the slowest rank's clock."""
    import torch

    def sync():
        br._sync()

    br.drain()
    sync()
    if dist_on:
        import torch.distributed as dist

        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(frames):
        br.step()
    br.drain()
    sync()
    if dist_on:
        dist.barrier()
    return frames / max_over_ranks(time.perf_counter() - t0, br.dev, dist_on)


def autotune_split(make, height, world, dist_on, frames=80, rounds=2, warm_seconds=0.25, candidates=None,
                   inflights=(2, 3)):
    """Sort-first load balancing on the hardware: every candidate (display-band size, frames in flight)
    (split_candidates) is built (make(display_rows, inflight) -> BandRenderer) and timed over `rounds`
    interleaved rounds of `frames` frames (the best round counts, so a clock ramp or a noisy round does not
    decide); the fastest wins, ties going to the more even split and fewer frames in flight. Every rank
    computes the same max-over-ranks rates, so every rank picks the same candidate without a broadcast.
    Returns ((display_rows, inflight), [(display_rows, inflight, frames/s), ...])."""
    cands = candidates or split_candidates(height, world, inflights=inflights)
    brs = []
    for d, k in cands:
        br = make(d, k)
        br.warm()
        brs.append(br)
    t_end = time.perf_counter() + warm_seconds  # the GPU's clock ramp out of idle, before any measurement
    while True:
        for _ in range(20):
            brs[0].step()
        brs[0].drain()
        if max_over_ranks(t_end - time.perf_counter(), brs[0].dev, dist_on) <= 0:
            break
    best = [0.0] * len(cands)
    for _ in range(rounds):
        for i, br in enumerate(brs):
            best[i] = max(best[i], measure_fps(br, frames, dist_on))
    for br in brs:
        br.close()
    pick = max(range(len(cands)), key=lambda i: (best[i], -cands[i][0], -cands[i][1]))
    return cands[pick], [(d, k, f) for (d, k), f in zip(cands, best)]


def rebalance_sizes(bands, ms, min_rows=32):
    """Sender bands re-cut in proportion to their measured row rates (rows / ms of each rank's render alone), the
    display band kept: the slowest sender sets the whole job's rate, so rows move from slow bands (dense geometry,
    the bottom of the frame) to fast ones. Every band keeps at least `min_rows` rows; largest remainders round.
    Deterministic, so every rank computes the same sizes from the same gathered times."""
    sizes = [b - a for a, b in bands]
    d, rest = sizes[0], sum(sizes[1:])
    rates = [sizes[r] / max(float(ms[r]), 1e-9) for r in range(1, len(sizes))]
    ideal = [rest * x / sum(rates) for x in rates]
    new = [max(min_rows, int(v)) for v in ideal]
    order = sorted(range(len(new)), key=lambda i: -(ideal[i] - int(ideal[i])))
    k = 0
    while sum(new) != rest and k < 10 * len(new) + rest:  # hand out (or take back) the remaining rows one at a time
        i = order[k % len(new)]
        if sum(new) < rest:
            new[i] += 1
        elif new[i] > min_rows:
            new[i] -= 1
        k += 1
    return [d] + new if sum(new) == rest else sizes


def rebalance_split(make, display_rows, inflight, dist_on, frames=80, rounds=2, warm_seconds=0.25):
    """One load-balancing step after autotune_split (band heights from the measured per-band time):
    every rank times its band's render alone, the times are all-gathered, the sender bands are re-cut by
    rebalance_sizes, and the re-cut split is kept only if it measures faster (max-over-ranks frames/s, interleaved
    rounds). Returns (display_rows or the list of band sizes, log)."""
    import torch

    br = make(display_rows, inflight)
    br.warm()
    ms = br.render_only_ms(frames=frames)
    world = len(br.bands)
    if dist_on:
        import torch.distributed as dist

        t = [torch.zeros(1, dtype=torch.float64, device=br.dev) for _ in range(world)]
        dist.all_gather(t, torch.tensor([ms], dtype=torch.float64, device=br.dev))
        times = [float(x.item()) for x in t]
    else:
        times = [ms] * world
    sizes = rebalance_sizes(br.bands, times)
    if sizes == [b - a for a, b in br.bands]:
        br.close()
        return display_rows, {"render_ms": times, "resplit": None}
    br2 = make(tuple(sizes), inflight)
    br2.warm()
    t_end = time.perf_counter() + warm_seconds
    while True:
        for _ in range(20):
            br.step()
        br.drain()
        if max_over_ranks(t_end - time.perf_counter(), br.dev, dist_on) <= 0:
            break
    best = [0.0, 0.0]
    for _ in range(rounds):
        for i, b in enumerate((br, br2)):
            best[i] = max(best[i], measure_fps(b, frames, dist_on))
    br.close()
    br2.close()
    log = {"render_ms": times, "resplit": sizes, "fps": {"autotuned": best[0], "resplit": best[1]}}
    return (tuple(sizes) if best[1] > best[0] else display_rows), log


def verify_assembly(br, scene, dist_on, frames=1, agree=True):
    """N > 1 parity in the bench itself: `frames` frames through the band exchange back to back (with several frames
    in flight every communicator and stream is exercised at once), and on the display rank the last assembled frame
    against the same frame rendered whole by one context on that GPU (bit for bit: a band context's pixels are the
    full frame's). With agree, every rank learns the outcome (a max over ranks); without, the
    caller agrees on "bad" (guarded() does, together with any exception). Returns a dict for the bench line's assembly
    object."""
    import numpy as np
    from trident_raster import raster, scenes

    for _ in range(frames):
        br.step()
    br.drain()
    br._sync(check=True)  # bounded, and every band lossless (the display sees the senders' status too)
    bad = 0.0
    note = "not the display rank"
    if br.rank == 0:
        got = br.assembled_frame().cpu().numpy().view(np.uint8).reshape(scene.height, scene.width, 4)
        with raster.TriRaster(scene.width, scene.height, device=br.dev.index) as r:
            scenes.load_scene(r, scene)
            r.render_frame()
            want, _ = r.readback(depth=False)
        diff = int((got != want).any(-1).sum())
        bad = float(diff)
        note = f"{diff} of {scene.width * scene.height} pixels differ from the one-context frame"
    if agree:
        bad = max_over_ranks(bad, br.dev, dist_on)
    return {"bit_exact": bad == 0.0, "detail": note, "bad": bad, "frames": frames}


def guarded_call(what, fn, device, dist_on, rank=0, bad=lambda out: 0.0):
    """Run fn() on every rank; an exception on any rank (a failed or timed-out native exchange: every wait is
    bounded) or a nonzero bad(out) is agreed over ranks in ONE collective after fn, and every rank then returns
    (ok, out or the failure detail) together, so the ranks' collective sequences stay aligned. fn's own collectives
    must not depend on the outcome."""
    try:
        out, err = fn(), None
    except Exception as e:  # noqa: BLE001 - any failure of the native path is reported and replaced
        out, err = None, f"{what}: {type(e).__name__}: {str(e)[:200]}"
        print(f"bench.py: rank {rank}: {err}", file=sys.stderr, flush=True)
    mine = 1e30 if err else float(bad(out))
    worst = max_over_ranks(mine, device, dist_on)
    if worst == 0.0:
        return True, out
    if err:
        return False, err
    if mine and isinstance(out, dict) and "detail" in out:
        return False, f"{what}: {out['detail']}"
    return False, f"{what}: failed on another rank ({worst:g})"


def timed_run(br, steps, warmup, dist_on, stage_timing=True, event_frames=256, warm_seconds=0.25):
    """Time exactly `steps` frames (no per-kernel events inside the timed region), then, outside it,
    a separate pass of `event_frames` frames with HIP events around every kernel of every frame:
    the per-kernel durations (roofline.kernel_ms) rest on that many samples, not on the few frames a
    short timed run would leave.

    Warm-up: `warmup` frames, back-to-back frames for at least `warm_seconds` of wall time, then batches
    of `steps` frames until two consecutive batches agree within 2 % (at most 8). The
    GPU leaves its idle clock state only after several ms of continuous work: after the scene upload
    (seconds of host work) 5 warm-up frames (0.6 ms) left the first timed frames at low clocks, and a
    20-frame run measured 0.134-0.140 ms/frame against 0.113-0.118 for the same frames after 50 ms of
    work (tools/step_timing.py, profiles/round3/step_timing.log). Nothing is removed from the timed
    region; it only starts at the clock every later frame runs at. Returns (seconds, timing, frames
    the warm-up ran)."""
    import torch

    br.warm()  # first frame per context sizes the internal queues (re-renders after TRI_E_OVERFLOW)
    t0 = time.perf_counter()
    for _ in range(max(warmup, 1)):
        br.step()
    br.drain()
    br._sync(check=True)  # (N > 1: a lossy band fails here, before any frame is counted)
    el = time.perf_counter() - t0
    # every rank runs the same number of frames (each one ends in a collective): the extra frames that
    # fill warm_seconds at the rate just measured, the maximum over ranks
    extra = 0 if el >= warm_seconds else min(int((warm_seconds - el) / (el / max(warmup, 1))) + 1, 100000)
    extra = int(max_over_ranks(float(extra), br.dev, dist_on))
    for _ in range(extra):
        br.step()
    # then batches of `steps` frames until two consecutive batches agree within 2 % (at most 8 batches):
    # the clock has settled at the rate the timed frames will run at
    batch, prev = max(steps, 20), None
    for _ in range(8):
        br.drain()
        br._sync()
        tb = time.perf_counter()
        for _ in range(batch):
            br.step()
        br.drain()
        br._sync()
        cur = max_over_ranks(time.perf_counter() - tb, br.dev, dist_on)
        extra += batch
        if prev is not None and abs(cur - prev) <= 0.02 * prev:
            break
        prev = cur
    n_warm = max(warmup, 1) + extra
    br.drain()
    br.synchronize()
    br._sync(check=True)
    if dist_on:
        import torch.distributed as dist

        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        br.step()
    br.drain()
    br._sync()  # (the native exchange's bounded wait, then the device; no flag read inside the timed region)
    if dist_on:
        dist.barrier()
    dt = time.perf_counter() - t0
    br.synchronize()  # surfaces TRI_E_OVERFLOW if any timed frame overflowed
    timing = None
    if stage_timing:  # per-kernel durations: context 0 alone, frames back to back without overlap
        br.r.set_timing(True, 1)
        for _ in range(event_frames):
            br.step(first_only=True)
        br.drain()
        timing = br.r.timing()
        br.r.set_timing(False)
    return max_over_ranks(dt, br.dev, dist_on), timing, n_warm


# Trident-Forge's editor frame: the Scene and Game viewport panels of the reference's own
# screenshot (Screenshots/Screenshot1.png: 992 x 1078 and 1064 x 1078 inside a 2559 x 1439 window, the extent the
# swapchain blit fills; tests/test_reference_frame.py crops the same panels)
FORGE_PANELS = {"viewports": ((2, 1064, 1078), (1, 992, 1078)), "present": (2559, 1439)}
FORGE_4K = {"viewports": ((1, 3840, 2160),), "present": (3840, 2160)}


def forge_frame(layout, frames=200, warm_seconds=0.25, frames_in_flight=1):
    """The frame Forge runs, through the engine API rather than the C-ABI: RenderCommand::DrawFrame on the
    Trident::Renderer shim (trident_app) with C3's 1M-triangle grid as one mesh entity, C3's sun and four point
    lights, the editor camera on the Scene viewport and a ready runtime camera on the Game viewport, the cubemap found
    by Init's discovery, and the present blit of the primary viewport (Renderer.cpp:733-837, :5208-5221, :5346-5361).
    Every DrawFrame gathers the draws, packs the uniform block per viewport, renders each viewport, blits, and waits
    for the previous frame first (the reference's fence, :752-772). Returns frames/s (DrawFrames completed per second)
    and the host cost of one DrawFrame: with the GPU idle (the engine's own work plus the launches) and as the
    renderer's GetFrameTimingStats record it in the loop (which includes the wait for the previous frame).
    frames_in_flight: Renderer::SetFramesInFlight — 1 is the reference's pacing; more keep that many targets per
    viewport so the next frames' front end overlaps this frame's raster, as the C-ABI line's contexts do."""
    from trident_raster import app, scenes

    s = build_scene("c3")
    a = app.TridentApp()
    try:
        a.set_assets_dir(scenes.ASSETS_DIR)
        a.set_frames_in_flight(frames_in_flight)
        mi = a.append_mesh(s.vertices, s.indices, base_color=(1.0, 1.0, 1.0, 1.0), metallic=0.1, roughness=0.6)
        a.add_mesh_entity("none", mi)
        a.add_light("directional", direction=(-0.5, -1.0, -0.3), intensity=3.0)
        for k, (px, py) in enumerate([(-3.0, 1.5), (3.0, 1.5), (-3.0, -1.5), (3.0, -1.5)]):
            a.add_light("point", position=(px, py, -2.5), color=(1.0, 0.9 - 0.1 * k, 0.7 + 0.1 * k),
                        intensity=3.0 + k, range=8.0)
        a.set_camera("editor", (0.0, 0.0, 0.0), (0.0, 0.0, 0.0), fov=60.0, near=0.1, far=1000.0)
        a.set_camera("runtime", (0.3, -0.2, 0.5), (4.0, 6.0, 0.0), fov=60.0, near=0.1, far=1000.0)
        for vid, w, h in layout["viewports"]:  # the last one set is the active (primary) viewport
            a.set_viewport(vid, w, h)
        a.set_present_extent(*layout["present"])
        a.draw_frame()
        a.finish_frame()
        t_end = time.perf_counter() + warm_seconds
        while time.perf_counter() < t_end:
            a.draw_frame()
        a.finish_frame()
        idle = []
        for _ in range(20):  # DrawFrame's host work with nothing to wait for
            a.finish_frame()
            t0 = time.perf_counter()
            a.draw_frame()
            idle.append((time.perf_counter() - t0) * 1e3)
        a.finish_frame()
        t0 = time.perf_counter()
        for _ in range(frames):
            a.draw_frame()
        a.finish_frame()
        dt = time.perf_counter() - t0
        timing = a.frame_timing()
        idle.sort()
        px = sum(w * h for _, w, h in layout["viewports"])
        return {"frames_per_s": frames / dt, "ms_per_frame": dt * 1e3 / frames,
                "viewports": [[w, h] for _, w, h in layout["viewports"]], "present": list(layout["present"]),
                "mpix_rendered_per_s": frames / dt * px / 1e6, "frames": frames,
                "host_ms_per_drawframe_idle_gpu": idle[len(idle) // 2],
                "drawframe_ms_avg_frame_timing_stats": timing["avg_ms"],
                "triangles": s.triangles, "frames_in_flight": frames_in_flight,
                "path": "RenderCommand::DrawFrame (Trident::Renderer shim, trident_app) -> tri_raster C-ABI"}
    finally:
        a.close()


def device_copy_gbs(device, nbytes=1 << 29, reps=10):
    """Measured HBM bandwidth of a device-to-device copy (read + write bytes per second), the practical
    ceiling next to the 8 TB/s spec peak."""
    import torch

    a = torch.empty(nbytes, dtype=torch.uint8, device=device)
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(reps):
        b.copy_(a)
    torch.cuda.synchronize(device)
    dt = time.perf_counter() - t0
    del a, b
    return 2.0 * nbytes * reps / dt / 1e9


def effective_cpus(cgroup_root="/sys/fs/cgroup"):
    """CPUs this process can use at once: min(affinity mask, cgroup v2 cpu.max quota / period,
    rounded up), falling back to the cgroup v1 cfs files. {"effective", "affinity", "quota"}; quota is
    None when unlimited or unreadable."""
    import math

    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count() or 1
    quota = None
    try:
        with open(os.path.join(cgroup_root, "cpu.max")) as f:
            q, period = f.read().split()[:2]
        if q != "max" and float(period) > 0:
            quota = math.ceil(float(q) / float(period))
    except (OSError, ValueError):
        try:
            with open(os.path.join(cgroup_root, "cpu", "cpu.cfs_quota_us")) as f:
                q = float(f.read())
            with open(os.path.join(cgroup_root, "cpu", "cpu.cfs_period_us")) as f:
                period = float(f.read())
            if q > 0 and period > 0:
                quota = math.ceil(q / period)
        except (OSError, ValueError):
            pass
    eff = max(1, min(affinity, quota) if quota else affinity)
    return {"effective": eff, "affinity": affinity, "quota": quota}


def cpu_baseline(scene, seconds):
    """The CPU oracle (a multithreaded C++ port of the same pipeline) on this host's cores, over a
    bounded sample of whole frames of the same workload (lavapipe is absent on this image)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py

    # every CPU this process may actually run on ("all host cores, core count stated"):
    # os.cpu_count() is the whole machine's, the job's share is its affinity mask and cgroup CPU quota
    host_cpus = os.cpu_count() or 1
    cpus = effective_cpus()
    threads = cpus["effective"]
    oracle_py.render(scene, threads=threads)  # warm-up frame (page-in, allocator)
    n, t0 = 0, time.perf_counter()
    while True:
        oracle_py.render(scene, threads=threads)
        n += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "frames/s", "cores": threads, "host_cpus": host_cpus,
            "affinity_cpus": cpus["affinity"], "cgroup_quota_cpus": cpus["quota"], "kind": "port",
            "sample": f"{n} full {scene.width}x{scene.height} frame(s) of {scene.name} "
                      f"({scene.triangles} tris) rendered by oracle/tri_oracle.cpp, {dt:.1f} s"}


PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_summary.json")


def pmc_kernel(workload, kernel, path=PMC_SUMMARY):
    """Per-launch PMC means of one kernel from the committed rocprofv3 summary (profiles/pmc_summary.json,
    written by tools/prof_summary.py from tools/profile.sh's passes), or None. The file must travel with the
    tree to the GPU box (.gpurunignore may not exclude it: round 4 lost roofline.traffic that way), so a
    missing or unreadable summary, or one without this workload's kernel, is reported on stderr."""
    try:
        with open(path) as f:
            entry = json.load(f).get(workload, {}).get(kernel)
    except (OSError, ValueError) as e:
        print(f"bench.py: WARNING: no PMC summary ({path}: {e}); roofline.traffic and roofline_valu will be null",
              file=sys.stderr, flush=True)
        return None
    if entry is None:
        print(f"bench.py: WARNING: {path} has no {kernel} entry for {workload}; roofline.traffic and roofline_valu "
              "will be null", file=sys.stderr, flush=True)
    return entry


# CDNA4 VALU issue: a wave64 vector instruction occupies its SIMD for 2 cycles (MI355X_MICROARCH.md),
# 256 CUs x 4 SIMDs, 2.4 GHz peak engine clock.
VALU_PEAK_WAVE_INSTS = 1024 * 2.4e9 / 2


def valu_roofline(pmc, kernel_ms):
    """The bound that binds k_raster: SQ_INSTS_VALU (wave instructions per launch, PMC) over the live
    kernel duration, against the chip's wave-instruction issue rate."""
    if not pmc or "SQ_INSTS_VALU" not in pmc or not kernel_ms:
        return None
    insts = float(pmc["SQ_INSTS_VALU"])
    achieved = insts / (kernel_ms * 1e-3)
    return {"bound": "valu", "kernel": "k_raster", "valu_wave_insts_per_launch": insts,
            "achieved": achieved / 1e9, "peak": VALU_PEAK_WAVE_INSTS / 1e9, "unit": "G wave-instructions/s",
            "frac": achieved / VALU_PEAK_WAVE_INSTS,
            "source": "profiles/pmc_summary.json SQ_INSTS_VALU / roofline.kernel_ms"}


def valu_floor_frac(pmc, raster_bytes):
    """The HBM fraction k_raster could reach if it ran at the VALU issue peak: its algorithmic bytes over the
    time its SQ_INSTS_VALU take at VALU_PEAK_WAVE_INSTS (the cap the VALU work alone puts on roofline.frac)."""
    if not pmc or "SQ_INSTS_VALU" not in pmc:
        return None
    floor_s = float(pmc["SQ_INSTS_VALU"]) / VALU_PEAK_WAVE_INSTS
    return raster_bytes / floor_s / 1e9 / HBM_PEAK_GBS


def stage_ms(timing):
    """Mean per-stage milliseconds of the event pass (zeros when stage timing is off)."""
    keys = ("ms_vertex", "ms_shadow", "ms_setup", "ms_raster", "ms_frame")
    if not timing or not timing.get("frames"):
        return {k: 0.0 for k in keys}
    n = float(timing["frames"])
    return {k: timing[k] / n for k in keys}


def rendering_rank_stage(br, timing, dist_on):
    """(stage ms, kernel samples, band rows) of the rank whose kernels the line describes: this rank's own, or, when
    the display rank 0 only assembles (a band of 0 rows, no kernels of its own), rank 1's, broadcast. Every rank calls
    it at the same point (the broadcast is a collective)."""
    stage = stage_ms(timing)
    samples = int(timing["frames"]) if timing else 0
    if not dist_on or br.bands[0][1] > br.bands[0][0]:
        return stage, samples, br.rows
    import torch
    import torch.distributed as dist

    keys = list(stage)
    t = torch.tensor([stage[k] for k in keys] + [samples, br.rows], dtype=torch.float64, device=br.dev)
    dist.broadcast(t, src=1)
    v = t.tolist()
    return dict(zip(keys, v[:len(keys)])), int(v[-2]), int(v[-1])


def skybox_name(scene):
    sky = scene.skybox
    if sky is None:
        return "none"
    if sky.shape[1] == 1:
        return "solid 0x808080 fallback cubemap (CreateSolidColor)"
    return f"reference Trident-Forge/Assets/Skyboxes PNG faces ({sky.shape[1]}^2, assets/Skyboxes)"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--warm-seconds", type=float, default=0.25,
                    help="untimed back-to-back frames before the timed region (at least --warmup frames): the "
                         "GPU's clock ramp out of idle takes a few ms")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--sim-world", type=int, default=0,
                    help="diagnostics (1 GPU, no collective): render only band --sim-rank of an N-way split")
    ap.add_argument("--sim-rank", type=int, default=0)
    ap.add_argument("--sim-extra-streams", type=int, default=0,
                    help="diagnostics: streams created (and kept) before the renderer, as a multi-GPU run's "
                         "collective libraries create theirs (HIP maps streams onto the process's hardware queues)")
    ap.add_argument("--sim-codec", choices=("none", "bgr24", "dbp"), default="none",
                    help="with --sim-world: every frame also packs this rank's band (sim rank > 0) or decodes the other "
                         "ranks' bands (sim rank 0, the display), on the frame's stream")
    ap.add_argument("--sim-display-rows", default=None,
                    help="diagnostics: the simulated split's display band (rank 0) size, the others sharing the rest; "
                         "or every band's size, comma-separated")
    ap.add_argument("--inflight", type=int, default=None,
                    help="frames in flight per rank (contexts taking frames in turn, one stream each); default per "
                         "config (DEFAULT_INFLIGHT)")
    ap.add_argument("--assembly", choices=("gather", "allgather"), default="gather",
                    help="N > 1: bands gathered onto the display rank 0 (default) or all-gathered onto every rank")
    ap.add_argument("--pack", choices=("auto", "dbp", "bgr24", "off"), default="auto",
                    help="N > 1 gather: when tri_frame_alpha proves every alpha byte equal, bands travel in the delta "
                         "bit-plane format (auto, dbp) or as 3 bytes per pixel (bgr24); off: always 4 bytes")
    ap.add_argument("--exchange", choices=("native", "torch"), default="native",
                    help="N > 1 gather: the band exchange through the library's own RCCL communicator, one call per frame "
                         "(native), or through torch.distributed point-to-point calls (torch)")
    ap.add_argument("--split", default="auto",
                    help="N > 1 gather: 'auto' (time candidate display-band sizes on the hardware, keep the fastest), "
                         "'equal', or the display rank's row count")
    ap.add_argument("--inflight-candidates", default="2,3",
                    help="N > 1 with --split auto: the frames-in-flight counts the autotune tries")
    ap.add_argument("--watchdog-seconds", type=float, default=600.0,
                    help="N > 1: host-side deadline per phase (exit non-zero with every thread's stack instead of "
                         "hanging the job); 0 disables")
    ap.add_argument("--no-stage-timing", action="store_true",
                    help="diagnostics: no per-kernel HIP events in the timed loop (roofline fields become null)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    import torch

    torch.cuda.set_device(local)
    dist_on = world > 1
    if dist_on:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    scene = build_scene(args.config)

    def inflight_for(sc):
        return args.inflight or DEFAULT_INFLIGHT.get(sc.name.split("_")[0], 2)

    def make_renderer(sc, display_rows=None, inflight=None):
        return BandRenderer(sc, rank, world, local, assembly=args.assembly, inflight=inflight or inflight_for(sc),
                            display_rows=display_rows, pack=args.pack, exchange=args.exchange)

    def autotuned_split(sc):
        """((display_rows or None, frames in flight), the autotune log) for a config at this world size."""
        if world == 1 or args.assembly != "gather" or args.split == "equal":
            return (None, inflight_for(sc)), None
        if args.split != "auto":
            return (int(args.split), inflight_for(sc)), None
        inflights = tuple(int(k) for k in args.inflight_candidates.split(","))
        cands = split_candidates(sc.height, world, inflights=inflights, assemble_only=args.exchange == "native")
        (d, k), log = autotune_split(lambda d, k: make_renderer(sc, d, k), sc.height, world, dist_on,
                                     warm_seconds=args.warm_seconds, candidates=cands)
        if world > 2:  # then one rebalancing step of the sender bands from their measured render times
            d, rlog = rebalance_split(lambda d, k: make_renderer(sc, d, k), d, k, dist_on,
                                      warm_seconds=args.warm_seconds)
            log = {"candidates": log, "rebalance": rlog}
        return (d, k), log

    def fall_back_to_torch(why):
        print(f"WARNING: native band exchange failed ({why}); using torch.distributed", file=sys.stderr, flush=True)
        args.exchange = "torch"

    def guarded(what, fn, bad=lambda out: 0.0):
        return guarded_call(what, fn, torch.device("cuda", local), dist_on, rank, bad)

    def native_check(sc):
        """Before any autotune: the native exchange on the equal split, 3 frames in flight over 30 frames, bit-exact
        against the one-GPU frame; (ok, parity dict or failure detail)."""
        def run():
            b = make_renderer(sc, None, 3)
            try:
                b.warm()
                return verify_assembly(b, sc, dist_on, frames=30, agree=False)
            finally:
                b.close()
        ok, res = guarded("native exchange check", run, bad=lambda out: out["bad"])
        if ok:
            res["bit_exact"] = True
        return ok, res

    def choose_split(sc):
        """autotuned_split, with the native exchange verified first and the autotune itself guarded: a failure of
        either switches the run to the torch.distributed exchange before anything is timed."""
        if world > 1 and args.assembly == "gather" and args.exchange == "native" and not native_checked:
            arm_watchdog(args.watchdog_seconds, "native exchange check")
            ok, res = native_check(sc)
            native_checked.append(res)
            if not ok:
                fall_back_to_torch(res)
        arm_watchdog(args.watchdog_seconds * 2 if world > 1 else 0, f"split autotune ({sc.name})")
        if args.exchange == "native" and world > 1:
            ok, res = guarded("split autotune", lambda: autotuned_split(sc))
            if ok:
                return res
            fall_back_to_torch(res)
        return autotuned_split(sc)

    native_checked = []
    split_log = None
    inflight = inflight_for(scene)
    if args.sim_world and world == 1:
        extra_streams = [torch.cuda.Stream(torch.device("cuda", local)) for _ in range(args.sim_extra_streams)]
        br = BandRenderer(scene, args.sim_rank, 1, local, band_world=args.sim_world, inflight=inflight_for(scene),
                          display_rows=(None if args.sim_display_rows is None else
                                        tuple(int(v) for v in args.sim_display_rows.split(","))
                                        if "," in args.sim_display_rows else int(args.sim_display_rows)),
                          pack=args.pack)
        if args.sim_codec != "none":
            br.attach_sim_codec(args.sim_codec)
    else:
        (display_rows, inflight), split_log = choose_split(scene)
        br = make_renderer(scene, display_rows, inflight)
    parity = None
    if world > 1 and args.assembly == "gather":
        # the assembled frame at the chosen split must equal the one-GPU frame; the native exchange falls back to
        # torch.distributed's if it does not (or fails), and the line says so
        arm_watchdog(args.watchdog_seconds, "assembly parity")
        ok, parity = guarded("assembly parity", lambda: verify_assembly(br, scene, dist_on, frames=10, agree=False),
                             bad=lambda out: out["bad"])
        if not ok:
            parity = {"bit_exact": False, "detail": parity}
        else:
            parity["bit_exact"] = True
        if not parity["bit_exact"] and br.xfer is not None:
            fall_back_to_torch(parity["detail"])
            br.close()
            if display_rows == 0 or (isinstance(display_rows, tuple) and display_rows[0] == 0):
                display_rows = None  # the torch exchange has no assemble-only display: the equal split
            br = make_renderer(scene, display_rows, inflight)
            parity = verify_assembly(br, scene, dist_on)
            parity["native_failed"] = True
        if native_checked:
            parity["native_check_before_autotune"] = native_checked[0]
    arm_watchdog(args.watchdog_seconds if world > 1 else 0, "timed run")
    dt, timing, n_warm = timed_run(br, args.steps, args.warmup, dist_on, not args.no_stage_timing,
                                   warm_seconds=args.warm_seconds)
    fps = args.steps / dt
    W, H = scene.width, scene.height
    stats = br.r.frame_stats()
    latency = br.latency_ms()  # one frame end to end (render + gather), no overlap
    stage, samples, rrows = rendering_rank_stage(br, timing, dist_on)  # rrows: the band those kernels rendered
    assembly = None
    if world > 1:  # what sets the rate: the slowest rank's render alone vs the assembly alone (outside the timed region)
        br.check()  # every packed band kept its alpha and fitted its slots (lossless)
        render_ms = max_over_ranks(br.render_only_ms(), br.dev, dist_on)
        asm_ms = max_over_ranks(br.assembly_only_ms(), br.dev, dist_on)
        inbound = br.inbound_bytes() if rank == 0 else 0
        assembly = {"render_ms": render_ms, "assembly_ms": asm_ms, "inbound_bytes_per_frame": inbound,
                    "exchange": "native (tri_xfer)" if br.xfer is not None else "torch.distributed",
                    "rccl_communicators": br.xfer_comms if br.xfer is not None else None,
                    "parity_vs_one_gpu_frame": parity,
                    "band_format": br.codec.mode if br.codec is not None else "bgra32",
                    "dbp_slot_bytes": br.codec.slot if br.codec is not None and br.codec.mode == "dbp" else None,
                    "band_bytes_per_pixel": (br.codec.bytes_for(rrows * W) / (rrows * W)
                                             if br.codec is not None else 4), "frame_alpha": br.alpha,
                    "render_bound_fps": 1e3 / render_ms if render_ms > 0 else None,
                    "assembly_bound_fps": 1e3 / asm_ms if asm_ms > 0 else None,
                    "bound": "assembly" if asm_ms > render_ms else "render",
                    "display_renders": br.bands[0][1] > br.bands[0][0],
                    "note": "max over ranks; render and assembly each timed alone, back to back, outside the timed region"}
    elif args.sim_world > 1:  # one band of an N-way split on one GPU: the codec's cost per band
        assembly = {"sim_world": args.sim_world, "sim_rank": args.sim_rank, "frame_alpha": br.alpha,
                    "sim_codec": args.sim_codec,
                    "codec": br.codec_ms([y1 - y0 for y0, y1 in br.bands])}

    # roofline of the dominant kernel (k_raster = tile_raster_shade): its algorithmic bytes per
    # launch are the colour + depth it must store for its band (4 + 4 B per pixel),
    # divided by its mean duration from HIP events on the render stream (a separate event pass).
    raster_ms = stage["ms_raster"]
    frame_ms = dt / args.steps * 1e3  # whole-frame figure on the throughput clock
    raster_bytes = 8.0 * W * rrows
    achieved = raster_bytes / (raster_ms * 1e-3) / 1e9 if raster_ms > 0 else None
    frame_bytes = scene.algorithmic_bytes(rows=rrows)
    pmc = pmc_kernel(scene.name, "k_raster")
    traffic = None if pmc is None or "hbm_bytes_per_launch" not in pmc else pmc["hbm_bytes_per_launch"] * rrows / H

    secondary = {}
    if not args.no_secondary and args.config == "c3":
        # the other BASELINE.json GPU configs, same timing protocol, and C3's grid under a non-identity model matrix
        # (how every Forge entity arrives: Renderer.cpp:417-427), so the headline's identity-draw path has its
        # general-path cost beside it
        for key in ("c2", "c5", "c3trs"):
            s2 = build_scene(key)
            (d2, k2), log2 = choose_split(s2)
            arm_watchdog(args.watchdog_seconds if world > 1 else 0, f"secondary {key}")
            br2 = make_renderer(s2, d2, k2)
            # enough frames that the pipeline's fill and drain (about one frame latency, 50 us at C2, 280 us at C5)
            # stay under 1 % of the timed region whatever --steps the headline uses
            n2 = max(args.steps, 200) if key in ("c2", "c3trs") else max(args.steps, 100)
            dt2, t2, _ = timed_run(br2, n2, args.warmup, dist_on, warm_seconds=args.warm_seconds)
            fps2 = n2 / dt2
            st2, samples2, rows2 = rendering_rank_stage(br2, t2, dist_on)
            entry = {"frames_per_s": fps2, "mpix_per_s": fps2 * s2.width * s2.height / 1e6, "ms_per_frame": 1e3 / fps2,
                     "stage_ms": st2, "kernel_samples": samples2, "triangles": s2.triangles,
                     "algorithmic_bytes": s2.algorithmic_bytes(rows=rows2)}
            entry["frames_in_flight"] = k2
            entry["fragment_path"] = br2.r.frame_stats()["path"]  # tri_frame_stats.path (TRI_PATH_* bits)
            if world > 1:
                entry["bands"] = [y1 - y0 for y0, y1 in br2.bands]
                entry["split_autotune"] = log2
            if s2.shadow is not None:
                entry["shadow_map"] = f"{s2.shadow.size}^2 D32 pre-pass for the sun (tri_set_shadow, DESIGN.md 5d)"
            if s2.textures:
                entry["textures"] = f"{len(s2.textures)} x {s2.textures[0][1].shape[0]}^2 sRGB, bilinear REPEAT"
            secondary[s2.name] = entry
            br2.close()
            del br2
    if not args.no_secondary and args.config == "c3" and world == 1:
        # Forge's editor frame through the engine API: two panels + the present blit, and one 4K
        # viewport, beside the C-ABI line
        secondary["forge_editor_frame_c3_panels"] = forge_frame(FORGE_PANELS)
        secondary["forge_editor_frame_c3_4k"] = forge_frame(FORGE_4K)
        # the same frames with three targets per viewport in flight (Renderer::SetFramesInFlight(3))
        secondary["forge_editor_frame_c3_panels_3inflight"] = forge_frame(FORGE_PANELS, frames_in_flight=3)
        secondary["forge_editor_frame_c3_4k_3inflight"] = forge_frame(FORGE_4K, frames_in_flight=3)

    arm_watchdog(0, "")
    copy_gbs = device_copy_gbs(br.dev) if rank == 0 else None
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(scene, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": fps,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_frames_run": n_warm,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (procedural PCG32-seeded scene; reference Assimp assets absent)",
            "config": {"workload": scene.name, "width": W, "height": H, "triangles": scene.triangles,
                       "vertices": int(scene.vertices.shape[0]), "bin": stats["bin_size"],
                       "skybox": skybox_name(scene), "frames_in_flight": inflight,
                       "parallelism": (f"row-band x{world} + RCCL {'gather to rank 0' if args.assembly == 'gather' else 'all-gather'}"
                                       if world > 1 else "single GPU"),
                       "bands": [y1 - y0 for y0, y1 in br.bands] if world > 1 else None,
                       "split_autotune": split_log},
            "mpix_per_s": fps * W * H / 1e6,
            "latency_ms": latency,
            # the pipeline's fill and drain: one frame's latency beyond its share of the throughput clock, paid once
            # per timed region (0.05 ms of a 20-step C3 region is ~2.6 %, of a 200-step one ~0.3 %)
            "fill_drain_ms": latency - dt / args.steps * 1e3,
            # the contract prices k_raster against HBM; what actually binds it is VALU issue together with the
            # L1 gather path (the VALU floor alone caps this frac near 0.17), see roofline_valu
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS if achieved else None, "traffic": traffic,
                         "binding": "valu issue + TA/TD gather path (roofline_valu), not HBM bytes",
                         "valu_floor_frac": valu_floor_frac(pmc if rrows == H else None, raster_bytes),
                         "measured_copy_GBs": copy_gbs,
                         "kernel": "k_raster",
                         "kernel_ms": raster_ms, "kernel_samples": samples,
                         "algorithmic_bytes": raster_bytes,
                         "traffic_source": (None if traffic is None else
                                            f"profiles/pmc_summary.json k_raster: {pmc.get('hbm_read_method', '2 x FETCH_SIZE')}"
                                            " reads + WRITE_SIZE, per launch; the read counters are calibrated against"
                                            " known bytes for k_raster's 12-B / 16-B gather shapes in"
                                            " profiles/round3/fetch_calib.json (tools/fetch_calib.sh)")},
            # the PMC count is of a whole frame: no VALU roofline for a band
            "roofline_valu": valu_roofline(pmc if rrows == H else None, raster_ms),
            "frame_roofline": {"algorithmic_bytes": frame_bytes, "ms_per_frame": frame_ms,
                               "achieved_GBs": frame_bytes / (frame_ms * 1e-3) / 1e9 if frame_ms > 0 else None,
                               "frac": frame_bytes / (frame_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if frame_ms > 0 else None},
            "stage_ms": stage,
            "assembly": assembly,
            "frame_stats": stats,
            "secondary": secondary,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    arm_watchdog(args.watchdog_seconds if world > 1 else 0, "teardown")
    br.close()
    if dist_on:
        import torch.distributed as dist

        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
