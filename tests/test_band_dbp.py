"""The delta bit-plane band format: a lossless band transfer at a fraction of the 3-byte format's bytes.
CPU: the numpy restatement (tests/dbp_ref.py) round-trips and sizes the C3 frame's bands. GPU: tri_dbp_pack writes
the restatement's bytes exactly, tri_dbp_unpack inverts it bit for bit, and the flags report alpha and slot overflow."""
import os

import numpy as np
import pytest

import dbp_ref


def _image(h, w, seed=3, noise=6):
    """A smooth gradient with per-pixel noise: what a shaded band looks like to the format."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    b = (xx * 255 // max(w - 1, 1) + rng.integers(-noise, noise + 1, (h, w))) % 256
    g = (yy * 255 // max(h - 1, 1) + rng.integers(-noise, noise + 1, (h, w))) % 256
    r = ((xx + yy) % 256 + rng.integers(-noise, noise + 1, (h, w))) % 256
    return (b | (g << 8) | (r << 16) | (255 << 24)).astype(np.uint32).ravel()


@pytest.mark.parametrize("n", [1, 63, 64, 1000, 1024, 4095, 4096, 4097, 9000])
def test_ref_round_trip_ragged(n):
    px = _image(1, n, seed=n)
    st, maxb, over = dbp_ref.encode(px, 12448)
    assert not over and maxb <= 12448
    assert np.array_equal(dbp_ref.decode(st, n, 255, 12448), px)


def test_ref_overflow_and_worst_case():
    """Random pixels need the full 8 planes per channel: 160 + 64 * 192 B = 12448 per slot, the format's maximum
    (TRI_DBP_MAX_SLOT); a smaller slot overflows and stays undecoded."""
    rng = np.random.default_rng(0)
    px = (rng.integers(0, 1 << 24, 4096, dtype=np.uint32) | np.uint32(255 << 24))
    st, maxb, over = dbp_ref.encode(px, 12448)
    assert maxb == 12448 and not over
    assert np.array_equal(dbp_ref.decode(st, 4096, 255, 12448), px)
    st, _, over = dbp_ref.encode(px, 8192)
    assert over and not dbp_ref.decode(st, 4096, 255, 8192).any()


def test_ref_c3_band_ratio(oracle):
    """The C3 frame's 8 bands of 270 rows (C4's split): 1.4-1.5 B per pixel on average against the 3-byte format."""
    from trident_raster import scenes

    s = scenes.scene_c3_grid(1920, 1080, 354)  # the same scene at a quarter of the pixels (the oracle in seconds)
    col, _, _ = oracle.render(s)
    words = col.view(np.uint32).reshape(1080, 1920)
    band = words[:135].ravel()
    st, maxb, over = dbp_ref.encode(band, 12448)
    payload = sum(int(st[i * 12448:i * 12448 + 4].view(np.uint32)[0]) + 160 for i in range(len(st) // 12448))
    assert not over and payload / band.size < 2.0, payload / band.size
    assert np.array_equal(dbp_ref.decode(st, band.size, 255, 12448), band)


@pytest.mark.gpu
@pytest.mark.parametrize("n,slot", [(4096 * 3 + 77, 12448), (3840 * 270, 8192), (1000, 2240)])
def test_gpu_dbp_matches_reference_and_round_trips(n, slot):
    import torch
    from trident_raster import raster

    px = _image(1, n, seed=n)
    want, maxb, over = dbp_ref.encode(px, slot)
    assert not over
    dev = torch.device("cuda", 0)
    src = torch.from_numpy(px.view(np.int32)).to(dev)
    stream = torch.zeros(raster.dbp_bytes(n, slot), dtype=torch.uint8, device=dev)
    flags = torch.zeros(2, dtype=torch.int32, device=dev)
    raster.dbp_pack(src.data_ptr(), n, 255, stream.data_ptr(), slot, flags.data_ptr(), torch.cuda.current_stream().cuda_stream)
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    raster.dbp_unpack(stream.data_ptr(), n, 255, slot, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    f = flags.cpu().numpy()
    assert f[0] == 0 and f[1] == maxb
    got = stream.cpu().numpy()
    # every slot's header and payload bytes equal the restatement's (bytes past the payload are unspecified)
    for s in range(len(want) // slot):
        nb = 160 + int(want[s * slot:s * slot + 4].view(np.uint32)[0])
        assert np.array_equal(got[s * slot:s * slot + nb], want[s * slot:s * slot + nb]), f"slot {s}"
    assert np.array_equal(out.cpu().numpy().view(np.uint32), px)


@pytest.mark.gpu
def test_gpu_dbp_flags_overflow_and_alpha():
    import torch
    from trident_raster import raster

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(1)
    px = rng.integers(0, 1 << 24, 8192, dtype=np.uint32) | np.uint32(255 << 24)
    px[5000] &= 0x00FFFFFF  # one alpha byte 0
    src = torch.from_numpy(px.view(np.int32)).to(dev)
    stream = torch.zeros(raster.dbp_bytes(8192, 4096), dtype=torch.uint8, device=dev)
    flags = torch.zeros(2, dtype=torch.int32, device=dev)
    raster.dbp_pack(src.data_ptr(), 8192, 255, stream.data_ptr(), 4096, flags.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    f = flags.cpu().numpy()
    assert f[0] == 3 and f[1] == 12448  # alpha mismatch + overflow; the slots need the maximum
    # the status travels with the band: slot 1 (pixels 4096..8191) carries the alpha mark in header word 1
    hdr = stream.cpu().numpy().reshape(2, 4096)[:, :8].copy().view(np.uint32)
    assert hdr[0, 1] == 0 and hdr[1, 1] == 1, hdr
    want, _, _ = dbp_ref.encode(px, 4096, alpha=255)
    assert np.array_equal(want.reshape(2, 4096)[:, :8], stream.cpu().numpy().reshape(2, 4096)[:, :8])


@pytest.mark.gpu
def test_gpu_dbp_c3_band_round_trip_and_cost(oracle):
    """The full C3 frame (oracle) as 8 bands of 3840 x 270: every band round-trips bit for bit at the slot size the
    largest slot needs; the ratio and the pack / unpack time per band go to gpurun_out/dbp_c3.txt."""
    import torch
    from trident_raster import raster, scenes

    col, _, _ = oracle.render(scenes.scene_c3_grid())
    words = col.view(np.uint32).reshape(2160, 3840)
    dev = torch.device("cuda", 0)
    lines = []
    for r in range(8):
        band = np.ascontiguousarray(words[270 * r:270 * (r + 1)]).ravel()
        n = band.size
        src = torch.from_numpy(band.view(np.int32)).to(dev)
        flags = torch.zeros(2, dtype=torch.int32, device=dev)
        big = torch.zeros(raster.dbp_bytes(n, 12448), dtype=torch.uint8, device=dev)
        cs = torch.cuda.current_stream().cuda_stream
        raster.dbp_pack(src.data_ptr(), n, 255, big.data_ptr(), 12448, flags.data_ptr(), cs)
        torch.cuda.synchronize()
        slot = (int(flags[1].item()) + 15) // 16 * 16
        stream = torch.zeros(raster.dbp_bytes(n, slot), dtype=torch.uint8, device=dev)
        out = torch.zeros(n, dtype=torch.int32, device=dev)
        flags.zero_()
        reps = 50
        raster.dbp_pack(src.data_ptr(), n, 255, stream.data_ptr(), slot, flags.data_ptr(), cs)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[0].record()
        for _ in range(reps):
            raster.dbp_pack(src.data_ptr(), n, 255, stream.data_ptr(), slot, flags.data_ptr(), cs)
        ev[1].record()
        for _ in range(reps):
            raster.dbp_unpack(stream.data_ptr(), n, 255, slot, out.data_ptr(), cs)
        ev[2].record()
        torch.cuda.synchronize()
        tp = ev[0].elapsed_time(ev[1]) / reps * 1e3  # back-to-back launches on the stream (GPU time per band)
        tu = ev[1].elapsed_time(ev[2]) / reps * 1e3
        assert int(flags[0].item()) == 0
        assert np.array_equal(out.cpu().numpy().view(np.uint32), band), f"band {r}"
        lines.append(f"band {r}: slot {slot} B = {slot / 4096:.3f} B/px on the link ({raster.dbp_bytes(n, slot) / 1e6:.2f} MB), "
                     f"pack {tp:.1f} us, unpack {tu:.1f} us")
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/dbp_c3.txt", "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


@pytest.mark.gpu
def test_gpu_dbp_unpack_skips_overflowed_and_foreign_slots():
    """The decoder leaves a slot alone when its payload does not fit the slot (the sender's overflow) or its widths do
    not add up to its payload count (bytes that are not this format): no out-of-slot read, the band untouched."""
    import torch
    from trident_raster import raster

    dev = torch.device("cuda", 0)
    n, slot = 3 * 4096, 2048
    st = np.zeros(raster.dbp_bytes(n, slot), np.uint8)
    rng = np.random.default_rng(7)
    st[:] = rng.integers(0, 256, st.size, dtype=np.uint8)
    words = st.view(np.uint32)
    words[0] = 4096            # slot 0: payload larger than the slot
    words[slot // 4] = 64      # slot 1: 8 planes claimed, widths random (sum almost surely != 8)
    words[2 * slot // 4] = 0   # slot 2: empty payload but random widths
    src = torch.from_numpy(st).to(dev)
    out = torch.full((n,), 7, dtype=torch.int32, device=dev)
    raster.dbp_unpack(src.data_ptr(), n, 255, slot, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert bool((out == 7).all())


@pytest.mark.gpu
def test_gpu_dbp_unpack_bands_one_launch():
    """tri_dbp_unpack_bands: ragged bands (an empty one among them) packed one by one at one slot size, decoded by one
    launch into their rows of a frame: bit-exact, and the rows of the empty band untouched."""
    import torch
    from trident_raster import raster

    dev = torch.device("cuda", 0)
    cs = torch.cuda.current_stream().cuda_stream
    sizes = [4096 * 5 + 17, 0, 1000, 4096 * 2, 63]
    slot = 8192
    px = [_image(1, max(n, 1), seed=11 + k)[:n] for k, n in enumerate(sizes)]
    streams, flags = [], torch.zeros(2, dtype=torch.int32, device=dev)
    for p in px:
        st = torch.zeros(max(raster.dbp_bytes(p.size, slot), 16), dtype=torch.uint8, device=dev)
        if p.size:
            src = torch.from_numpy(p.view(np.int32).copy()).to(dev)
            raster.dbp_pack(src.data_ptr(), p.size, 255, st.data_ptr(), slot, flags.data_ptr(), cs)
        streams.append(st)
    frame = torch.full((sum(sizes) + 5,), 7, dtype=torch.int32, device=dev)
    offs = np.concatenate([[0], np.cumsum(sizes)])
    raster.dbp_unpack_bands([s.data_ptr() for s in streams], [frame.data_ptr() + 4 * int(o) for o in offs[:-1]],
                            sizes, 255, slot, cs)
    torch.cuda.synchronize()
    assert int(flags[0].item()) == 0
    got = frame.cpu().numpy().view(np.uint32)
    assert np.array_equal(got[:sum(sizes)], np.concatenate(px))
    assert (got[sum(sizes):] == 7).all()
