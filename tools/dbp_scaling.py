"""Codec cost against size on one GPU: tri_dbp_pack / tri_dbp_unpack and the 3-byte pair over 1..8 C3-like bands in
one launch (HIP events, back-to-back launches), to separate a launch's fixed latency from its per-pixel cost.
Writes gpurun_out/dbp_scaling.txt."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-renderer_amd", "python"))
from trident_raster import raster  # noqa: E402


def image(h, w, seed=3, noise=3):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    b = (xx * 255 // (w - 1) + rng.integers(-noise, noise + 1, (h, w))) % 256
    g = (yy * 255 // (h - 1) + rng.integers(-noise, noise + 1, (h, w))) % 256
    r = ((xx + yy) % 256 + rng.integers(-noise, noise + 1, (h, w))) % 256
    return (b | (g << 8) | (r << 16) | (255 << 24)).astype(np.uint32).ravel()


def main():
    dev = torch.device("cuda", 0)
    cs = torch.cuda.current_stream().cuda_stream
    lines = []
    base = image(270, 3840)
    for k in tuple(int(x) for x in os.environ.get("DBP_SIZES", "1,2,4,8").split(",")):
        px = np.tile(base, k)
        n = px.size
        src = torch.from_numpy(px.view(np.int32)).to(dev)
        flags = torch.zeros(2, dtype=torch.int32, device=dev)
        big = torch.zeros(raster.dbp_bytes(n, 12448), dtype=torch.uint8, device=dev)
        raster.dbp_pack(src.data_ptr(), n, 255, big.data_ptr(), 12448, flags.data_ptr(), cs)
        torch.cuda.synchronize()
        slot = (int(flags[1].item()) + 15) // 16 * 16
        st = torch.zeros(raster.dbp_bytes(n, slot), dtype=torch.uint8, device=dev)
        out = torch.zeros(n, dtype=torch.int32, device=dev)
        b3 = torch.zeros(3 * n, dtype=torch.uint8, device=dev)
        reps = 100
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
        for _ in range(10):
            raster.dbp_pack(src.data_ptr(), n, 255, st.data_ptr(), slot, flags.data_ptr(), cs)
        ev[0].record()
        for _ in range(reps):
            raster.dbp_pack(src.data_ptr(), n, 255, st.data_ptr(), slot, flags.data_ptr(), cs)
        ev[1].record()
        for _ in range(reps):
            raster.dbp_unpack(st.data_ptr(), n, 255, slot, out.data_ptr(), cs)
        ev[2].record()
        for _ in range(reps):
            raster.pack_bgr24(src.data_ptr(), b3.data_ptr(), n, 255, flags.data_ptr(), cs)
        ev[3].record()
        for _ in range(reps):
            raster.unpack_bgr24(b3.data_ptr(), out.data_ptr(), n, 255, cs)
        ev[4].record()
        torch.cuda.synchronize()
        t = [ev[i].elapsed_time(ev[i + 1]) / reps * 1e3 for i in range(4)]
        ok = bool(torch.equal(out, src))
        lines.append(f"{k} band(s) {n} px: dbp pack {t[0]:.1f} us unpack {t[1]:.1f} us | bgr24 pack {t[2]:.1f} us "
                     f"unpack {t[3]:.1f} us | slot {slot} round-trip {'ok' if ok else 'MISMATCH'}")
        print(lines[-1], flush=True)
    # the display GPU at N = 8: seven remote bands decoded by one launch
    n = base.size
    src = torch.from_numpy(base.view(np.int32)).to(dev)
    st = torch.zeros(raster.dbp_bytes(n, slot), dtype=torch.uint8, device=dev)
    raster.dbp_pack(src.data_ptr(), n, 255, st.data_ptr(), slot, flags.data_ptr(), cs)
    frame = torch.zeros(7 * n, dtype=torch.int32, device=dev)
    args = ([st.data_ptr()] * 7, [frame.data_ptr() + 4 * k * n for k in range(7)], [n] * 7, 255, slot, cs)
    for _ in range(10):
        raster.dbp_unpack_bands(*args)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(100):
        raster.dbp_unpack_bands(*args)
    ev[1].record()
    torch.cuda.synchronize()
    ok = bool(torch.equal(frame.view(7, n), src.expand(7, n)))
    lines.append(f"7 remote bands in one tri_dbp_unpack_bands launch: {ev[0].elapsed_time(ev[1]) / 100 * 1e3:.1f} us "
                 f"({'ok' if ok else 'MISMATCH'})")
    print(lines[-1], flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/dbp_scaling.txt", "w") as f:
        f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
