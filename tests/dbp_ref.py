"""TEST INFRASTRUCTURE: a numpy restatement of the delta bit-plane band format (band_codec.hip, include/tri_raster.h
tri_dbp_*), so the GPU stream's bytes are checked against an independent encoder and decoded by an independent
decoder. Not a product path."""
import numpy as np

SLOT_PIXELS, SEGMENT, HEADER = 4096, 1024, 160


def _zig(d):
    return np.where(d >= 0, 2 * d, -2 * d - 1).astype(np.uint32)


def encode(bgra, slot_bytes, alpha=None):
    """bgra: uint32 [n] (B8G8R8A8 words). Returns (stream uint8 [nslots * slot_bytes], max slot bytes, overflow).
    alpha: the promised alpha; a slot holding a pixel whose alpha differs carries 1 in header word 1 (the sender's
    status, which the display's decode reports)."""
    px = np.asarray(bgra, np.uint32).ravel()
    n = px.size
    nslots = (n + SLOT_PIXELS - 1) // SLOT_PIXELS
    out = np.zeros(nslots * slot_bytes, np.uint8)
    maxb, over = 0, False
    for s in range(nslots):
        hdr = np.zeros(HEADER // 4, np.uint32)
        planes = []
        for w in range(4):
            seg0 = (s * 4 + w) * SEGMENT
            if seg0 >= n:
                continue
            first = int(px[seg0]) & 0x00FFFFFF
            hdr[4 + 9 * w] = first
            widths = np.zeros(16, np.uint16)
            carry = first
            for k in range(16):
                i = seg0 + 64 * k + np.arange(64)
                v = px[np.minimum(i, n - 1)].astype(np.int64)
                prev = np.concatenate([[carry], v[:-1]])
                carry = int(v[63])
                wk = 0
                for c in range(3):
                    d = (((v >> (8 * c)) - (prev >> (8 * c))) & 0xFF).astype(np.int64)
                    d = np.where(d >= 128, d - 256, d)
                    z = _zig(d)
                    wc = int(z.max()).bit_length()
                    wk |= wc << (4 * c)
                    for j in range(wc):
                        bits = ((z >> j) & 1).astype(np.uint64)
                        planes.append(int((bits << np.arange(64, dtype=np.uint64)).sum()))
                widths[k] = wk
            hdr[4 + 9 * w + 1: 4 + 9 * w + 9] = widths.view(np.uint32)
        total = 8 * len(planes)
        hdr[0] = total
        sp = px[s * SLOT_PIXELS:(s + 1) * SLOT_PIXELS]
        hdr[1] = 1 if alpha is not None and bool(((sp >> 24) != alpha).any()) else 0
        nbytes = HEADER + total
        maxb = max(maxb, nbytes)
        slot = out[s * slot_bytes:(s + 1) * slot_bytes]
        if nbytes > slot_bytes:
            over = True
            slot[:8] = np.array([total, hdr[1]], np.uint32).view(np.uint8)
            continue
        slot[:HEADER] = hdr.view(np.uint8)
        if planes:
            slot[HEADER:HEADER + total] = np.array(planes, np.uint64).view(np.uint8)
    return out, maxb, over


def decode(stream, n, alpha, slot_bytes):
    """The inverse of encode: uint32 [n] B8G8R8A8 words (alpha restored); overflowed slots stay 0."""
    out = np.zeros(n, np.uint32)
    nslots = (n + SLOT_PIXELS - 1) // SLOT_PIXELS
    for s in range(nslots):
        slot = stream[s * slot_bytes:(s + 1) * slot_bytes]
        hdr = slot[:HEADER].view(np.uint32)
        if HEADER + int(hdr[0]) > slot_bytes:
            continue
        pay = slot[HEADER:].view(np.uint64) if slot_bytes > HEADER else np.zeros(0, np.uint64)
        off = 0
        for w in range(4):
            seg0 = (s * 4 + w) * SEGMENT
            widths = hdr[4 + 9 * w + 1: 4 + 9 * w + 9].view(np.uint16)
            carry = int(hdr[4 + 9 * w])
            for k in range(16):
                val = np.full(64, alpha << 24, np.int64)
                wk = int(widths[k])
                for c in range(3):
                    wc = (wk >> (4 * c)) & 15
                    z = np.zeros(64, np.int64)
                    for j in range(wc):
                        z |= ((pay[off] >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).astype(np.int64) << j
                        off += 1
                    d = np.where(z & 1, -((z + 1) >> 1), z >> 1)
                    ch = (np.cumsum(d) + ((carry >> (8 * c)) & 0xFF)) & 0xFF
                    val |= ch << (8 * c)
                i = seg0 + 64 * k + np.arange(64)
                ok = i < n
                out[i[ok]] = val[ok].astype(np.uint32)
                carry = int(val[63]) & 0x00FFFFFF
    return out
