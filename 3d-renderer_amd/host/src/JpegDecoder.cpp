// JpegDecoder.cpp — baseline and progressive JPEG for TextureLoader (Trident's stbi_load path,
// TextureLoader.cpp:290-304). stb_image is an un-vendored submodule of the reference; its published JPEG
// algorithm is restated here (JFIF / ITU T.81 decoding with stb's observable choices):
//   - Huffman-coded baseline (SOF0 / SOF1) and progressive (SOF2) frames, 8-bit samples, 1 or 3
//     components, any sampling factors 1..4, restart intervals, 8- and 16-bit quantisation tables;
//   - the integer IDCT of the IJG "islow" family with 12-bit fixed-point constants (rounded column pass
//     >> 10, row pass >> 17 with the +128 level shift folded into the rounding), results clamped to 0..255;
//   - chroma upsampling: 2x horizontal and 2x vertical by the 3:1 triangle filter ("fancy" upsampling),
//     2x2 by the separable form (vertical 3:1 sum, then horizontal (3 a + b + 8) >> 4), nearest
//     replication for other factor ratios;
//   - YCbCr -> RGB in 20-bit fixed point (1.402, 0.71414, 0.34414, 1.772), unless an Adobe APP14 marker
//     says "no transform" or the component ids are 'R', 'G', 'B';
//   - forced 4 channels: grey g -> (g, g, g, 255), colour -> (r, g, b, 255).
// Arithmetic coding, 12-bit samples, lossless and 4-component (CMYK / YCCK) files are rejected, as a
// failed stbi_load would be.
#include "trident/ImageDecoder.h"

#include <algorithm>
#include <array>
#include <cstring>

namespace Trident {
namespace Loader {

namespace {

// zig-zag order -> natural (row-major) position in the 8x8 block
constexpr uint8_t kDezigzag[64 + 15] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13,
    6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31,
    39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
    // a corrupt run past the end lands on the last coefficient
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

struct Huffman {
    // canonical code per length: codes of length L are [mincode[L], mincode[L] + count[L]), values follow
    uint16_t count[17] = {};
    int32_t maxcode[18] = {};
    int32_t valptr[17] = {};
    int32_t mincode[17] = {};
    uint8_t values[256] = {};
    bool defined = false;
    void build() {
        int32_t code = 0, k = 0;
        for (int l = 1; l <= 16; ++l) {
            valptr[l] = k;
            mincode[l] = code;
            code += count[l];
            k += count[l];
            maxcode[l] = count[l] ? code - 1 : -1;
            code <<= 1;
        }
        maxcode[17] = 0x7fffffff;
        defined = true;
    }
};

struct Component {
    int id = 0, h = 1, v = 1, tq = 0;
    int td = 0, ta = 0;     // Huffman table selectors of the current scan
    int bw = 0, bh = 0;     // blocks per line / column (padded to whole MCUs)
    int dc_pred = 0;
    std::vector<int16_t> coef;    // progressive: every block's coefficients (natural order)
    std::vector<uint8_t> pixels;  // bw*8 x bh*8 samples
};

struct Decoder {
    const uint8_t* p = nullptr;
    size_t n = 0, pos = 0;
    std::string err;
    uint16_t qt[4][64] = {};
    Huffman hdc[4], hac[4];
    std::vector<Component> comp;
    int width = 0, height = 0, hmax = 1, vmax = 1, mcux = 0, mcuy = 0;
    bool progressive = false;
    int restart_interval = 0;
    int adobe_transform = -1;  // APP14 transform flag (-1: no Adobe marker)
    bool jfif = false;         // an APP0 "JFIF" marker
    // entropy-coded segment reader
    uint32_t bitbuf = 0;
    int bitcnt = 0;
    bool hit_marker = false;
    int eobrun = 0;
    // current scan
    int ss = 0, se = 63, ah = 0, al = 0;
    std::vector<int> scomp;

    bool fail(const char* m) {
        if (err.empty()) err = m;
        return false;
    }
    int byte() { return pos < n ? p[pos++] : (hit_marker = true, 0); }
    int u16() {
        const int a = byte();
        return (a << 8) | byte();
    }

    void fill() {
        while (bitcnt <= 24) {
            int c = 0;
            if (!hit_marker) {
                if (pos >= n) {
                    hit_marker = true;
                } else {
                    c = p[pos];
                    if (c == 0xFF) {
                        const int nx = pos + 1 < n ? p[pos + 1] : 0xD9;
                        if (nx == 0x00) {
                            pos += 2;  // stuffed 0xFF
                        } else {
                            hit_marker = true;  // a marker ends the segment: feed zeros
                            c = 0;
                        }
                    } else {
                        ++pos;
                    }
                }
            }
            bitbuf |= (uint32_t)c << (24 - bitcnt);
            bitcnt += 8;
        }
    }
    int bits(int k) {  // k <= 16
        if (k == 0) return 0;
        fill();
        const int v = (int)(bitbuf >> (32 - k));
        bitbuf <<= k;
        bitcnt -= k;
        return v;
    }
    int bit() { return bits(1); }
    // F.2.2.1 EXTEND: a k-bit magnitude category value to its signed coefficient
    int receive_extend(int k) {
        if (k == 0) return 0;
        const int v = bits(k);
        return v < (1 << (k - 1)) ? v - (1 << k) + 1 : v;
    }
    int decode(const Huffman& h) {
        fill();
        int32_t code = 0;
        for (int l = 1; l <= 16; ++l) {
            code = (code << 1) | (int)(bitbuf >> 31);
            bitbuf <<= 1;
            --bitcnt;
            if (code <= h.maxcode[l]) return h.values[h.valptr[l] + code - h.mincode[l]];
        }
        return -1;  // corrupt
    }
    void reset_entropy() {
        bitbuf = 0;
        bitcnt = 0;
        hit_marker = false;
        eobrun = 0;
        for (Component& c : comp) c.dc_pred = 0;
    }
    // After an interval: skip to the RSTn marker (a corrupt stream resynchronises on the next one).
    bool restart() {
        bitbuf = 0;
        bitcnt = 0;
        while (pos + 1 < n && !(p[pos] == 0xFF && p[pos + 1] >= 0xD0 && p[pos + 1] <= 0xD7)) ++pos;
        if (pos + 1 >= n) return fail("missing restart marker");
        pos += 2;
        reset_entropy();
        return true;
    }

    bool read_dqt(int len) {
        const size_t end = pos + len;
        while (pos < end) {
            const int pq = byte(), t = pq & 15, prec = pq >> 4;
            if (t > 3 || prec > 1) return fail("bad DQT");
            for (int i = 0; i < 64; ++i) qt[t][kDezigzag[i]] = (uint16_t)(prec ? u16() : byte());
        }
        return pos == end || fail("bad DQT length");
    }
    bool read_dht(int len) {
        const size_t end = pos + len;
        while (pos < end) {
            const int tc = byte(), cls = tc >> 4, t = tc & 15;
            if (cls > 1 || t > 3) return fail("bad DHT");
            Huffman& h = cls ? hac[t] : hdc[t];
            int total = 0;
            for (int l = 1; l <= 16; ++l) total += (h.count[l] = (uint16_t)byte());
            if (total > 256) return fail("bad DHT counts");
            for (int i = 0; i < total; ++i) h.values[i] = (uint8_t)byte();
            h.build();
        }
        return pos == end || fail("bad DHT length");
    }
    bool read_sof(int len, bool prog) {
        progressive = prog;
        if (byte() != 8) return fail("only 8-bit JPEG samples are supported");
        height = u16();
        width = u16();
        const int nc = byte();
        if (width <= 0 || height <= 0) return fail("bad JPEG dimensions (DNL is not supported)");
        if (nc != 1 && nc != 3) return fail("only 1- and 3-component JPEGs are supported");
        if (len != 6 + 3 * nc) return fail("bad SOF length");
        if ((int64_t)width * height > (1 << 28)) return fail("JPEG too large");
        comp.assign(nc, Component{});
        for (Component& c : comp) {
            c.id = byte();
            const int hv = byte();
            c.h = hv >> 4;
            c.v = hv & 15;
            c.tq = byte();
            if (c.h < 1 || c.h > 4 || c.v < 1 || c.v > 4 || c.tq > 3) return fail("bad component");
            hmax = std::max(hmax, c.h);
            vmax = std::max(vmax, c.v);
        }
        mcux = (width + 8 * hmax - 1) / (8 * hmax);
        mcuy = (height + 8 * vmax - 1) / (8 * vmax);
        for (Component& c : comp) {
            c.bw = mcux * c.h;
            c.bh = mcuy * c.v;
            c.pixels.assign((size_t)c.bw * 8 * c.bh * 8, 0);
            if (progressive) c.coef.assign((size_t)c.bw * c.bh * 64, 0);
        }
        return true;
    }

    // ---- baseline block ----
    bool decode_block(Component& c, int16_t* out) {
        std::memset(out, 0, 64 * sizeof(int16_t));
        const int t = decode(hdc[c.td]);
        if (t < 0 || t > 16) return fail("bad Huffman code");
        c.dc_pred += receive_extend(t);
        out[0] = (int16_t)(c.dc_pred * qt[c.tq][0]);
        for (int k = 1; k < 64;) {
            const int rs = decode(hac[c.ta]);
            if (rs < 0) return fail("bad Huffman code");
            const int r = rs >> 4, s = rs & 15;
            if (s == 0) {
                if (r != 15) break;  // EOB
                k += 16;
                continue;
            }
            k += r;
            const int z = kDezigzag[k];
            out[z] = (int16_t)(receive_extend(s) * qt[c.tq][z]);
            ++k;
        }
        return true;
    }

    // ---- progressive (G.1.2) ----
    bool prog_dc(Component& c, int16_t* b) {
        if (ah == 0) {
            const int t = decode(hdc[c.td]);
            if (t < 0 || t > 16) return fail("bad Huffman code");
            c.dc_pred += receive_extend(t);
            b[0] = (int16_t)(c.dc_pred * (1 << al));
        } else if (bit()) {
            b[0] = (int16_t)(b[0] | (1 << al));
        }
        return true;
    }
    bool prog_ac_first(Component& c, int16_t* b) {
        if (eobrun > 0) {
            --eobrun;
            return true;
        }
        for (int k = ss; k <= se;) {
            const int rs = decode(hac[c.ta]);
            if (rs < 0) return fail("bad Huffman code");
            const int r = rs >> 4, s = rs & 15;
            if (s == 0) {
                if (r < 15) {
                    eobrun = (1 << r) - 1;
                    if (r) eobrun += bits(r);
                    break;
                }
                k += 16;
                continue;
            }
            k += r;
            b[kDezigzag[k]] = (int16_t)(receive_extend(s) * (1 << al));
            ++k;
        }
        return true;
    }
    bool prog_ac_refine(Component& c, int16_t* b) {
        const int p1 = 1 << al, m1 = -1 * (1 << al);
        auto refine = [&](int16_t& coef) {
            if (coef != 0 && bit() && (coef & p1) == 0) coef = (int16_t)(coef > 0 ? coef + p1 : coef + m1);
        };
        int k = ss;
        if (eobrun <= 0) {
            for (; k <= se;) {
                const int rs = decode(hac[c.ta]);
                if (rs < 0) return fail("bad Huffman code");
                int r = rs >> 4;
                const int s = rs & 15;
                int val = 0;
                if (s == 0) {
                    if (r < 15) {
                        eobrun = (1 << r);
                        if (r) eobrun += bits(r);
                        break;  // the rest of the band is refined below
                    }
                    // r == 15: skip 16 zero coefficients (refining non-zero ones on the way)
                } else {
                    val = bit() ? p1 : m1;
                }
                while (k <= se) {
                    int16_t& coef = b[kDezigzag[k]];
                    if (coef != 0) {
                        refine(coef);
                    } else {
                        if (r == 0) {
                            if (val) coef = (int16_t)val;
                            ++k;
                            break;
                        }
                        --r;
                    }
                    ++k;
                }
            }
        }
        if (eobrun > 0) {  // inside an EOB run: only refine the non-zero coefficients of the band
            for (; k <= se; ++k) refine(b[kDezigzag[k]]);
            --eobrun;
        }
        return true;
    }

    bool read_sos(int len) {
        const int ns = byte();
        if (ns < 1 || ns > 4 || len != 4 + 2 * ns) return fail("bad SOS");
        scomp.clear();
        for (int i = 0; i < ns; ++i) {
            const int id = byte(), t = byte();
            int ci = -1;
            for (size_t k = 0; k < comp.size(); ++k)
                if (comp[k].id == id) ci = (int)k;
            if (ci < 0) return fail("SOS names an unknown component");
            comp[ci].td = t >> 4;
            comp[ci].ta = t & 15;
            if (comp[ci].td > 3 || comp[ci].ta > 3) return fail("bad Huffman selector");
            scomp.push_back(ci);
        }
        ss = byte();
        se = byte();
        const int a = byte();
        ah = a >> 4;
        al = a & 15;
        if (progressive) {
            if (ss > se || se > 63 || (ss == 0 && se != 0) || (ss > 0 && ns != 1) || al > 13)
                return fail("bad progressive scan");
        } else if (ss != 0 || se != 63 || a != 0) {
            return fail("bad baseline scan");
        }
        for (int ci : scomp) {
            const Component& c = comp[ci];
            if ((!progressive || ss == 0) && ah == 0 && !hdc[c.td].defined) return fail("undefined DC table");
            if ((!progressive || ss > 0) && !hac[c.ta].defined) return fail("undefined AC table");
        }
        return true;
    }

    bool decode_scan() {
        reset_entropy();
        int16_t tmp[64];
        auto block = [&](Component& c, int bx, int by) -> bool {
            if (!progressive) {
                if (!decode_block(c, tmp)) return false;
                idct_block(tmp, c.pixels.data() + (size_t)by * 8 * c.bw * 8 + (size_t)bx * 8, c.bw * 8);
                return true;
            }
            int16_t* b = c.coef.data() + ((size_t)by * c.bw + bx) * 64;
            if (ss == 0) return prog_dc(c, b);
            return ah == 0 ? prog_ac_first(c, b) : prog_ac_refine(c, b);
        };
        int todo = restart_interval ? restart_interval : 0x7fffffff;
        if (scomp.size() == 1) {  // non-interleaved: blocks of the component's own (unpadded) extent
            Component& c = comp[scomp[0]];
            const int w = (width * c.h + 8 * hmax - 1) / (8 * hmax), h = (height * c.v + 8 * vmax - 1) / (8 * vmax);
            for (int by = 0; by < h; ++by)
                for (int bx = 0; bx < w; ++bx) {
                    if (!block(c, bx, by)) return false;
                    if (--todo == 0 && !(by == h - 1 && bx == w - 1)) {
                        if (!restart()) return false;
                        todo = restart_interval;
                    }
                }
        } else {
            for (int my = 0; my < mcuy; ++my)
                for (int mx = 0; mx < mcux; ++mx) {
                    for (int ci : scomp) {
                        Component& c = comp[ci];
                        for (int y = 0; y < c.v; ++y)
                            for (int x = 0; x < c.h; ++x)
                                if (!block(c, mx * c.h + x, my * c.v + y)) return false;
                    }
                    if (--todo == 0 && !(my == mcuy - 1 && mx == mcux - 1)) {
                        if (!restart()) return false;
                        todo = restart_interval;
                    }
                }
        }
        // skip to the next marker
        while (pos + 1 < n && !(p[pos] == 0xFF && p[pos + 1] != 0x00 && !(p[pos + 1] >= 0xD0 && p[pos + 1] <= 0xD7))) ++pos;
        return true;
    }

    // IJG islow IDCT with 12-bit constants: column pass (>> 10 with rounding), row pass (>> 17, the +128
    // level shift folded into the rounding term), clamp to 0..255. `in` is dequantised, natural order.
    static void idct_block(const int16_t* in, uint8_t* out, int stride) {
        auto f2f = [](float x) { return (int)(x * 4096.0f + 0.5f); };
        const int c0541 = f2f(0.5411961f), c0765 = f2f(0.765366865f), c1847 = f2f(-1.847759065f);
        const int c1175 = f2f(1.175875602f), c0298 = f2f(0.298631336f), c2053 = f2f(2.053119869f),
                  c3072 = f2f(3.072711026f), c1501 = f2f(1.501321110f), c0899 = f2f(-0.899976223f),
                  c2562 = f2f(-2.562915447f), c1961 = f2f(-1.961570560f), c0390 = f2f(-0.390180644f);
        int v[64];
        auto idct1d = [&](int s0, int s1, int s2, int s3, int s4, int s5, int s6, int s7, int& t0, int& t1, int& t2,
                          int& t3, int& x0, int& x1, int& x2, int& x3) {
            int p2 = s2, p3 = s6;
            int p1 = (p2 + p3) * c0541;
            t2 = p1 + p3 * c1847;
            t3 = p1 + p2 * c0765;
            p2 = s0;
            p3 = s4;
            t0 = (p2 + p3) * 4096;
            t1 = (p2 - p3) * 4096;
            x0 = t0 + t3;
            x3 = t0 - t3;
            x1 = t1 + t2;
            x2 = t1 - t2;
            t0 = s7;
            t1 = s5;
            t2 = s3;
            t3 = s1;
            p3 = t0 + t2;
            int p4 = t1 + t3;
            p1 = t0 + t3;
            p2 = t1 + t2;
            const int p5 = (p3 + p4) * c1175;
            t0 = t0 * c0298;
            t1 = t1 * c2053;
            t2 = t2 * c3072;
            t3 = t3 * c1501;
            p1 = p5 + p1 * c0899;
            p2 = p5 + p2 * c2562;
            p3 = p3 * c1961;
            p4 = p4 * c0390;
            t3 += p1 + p4;
            t2 += p2 + p3;
            t1 += p2 + p4;
            t0 += p1 + p3;
        };
        for (int i = 0; i < 8; ++i) {  // columns
            const int16_t* d = in + i;
            int* o = v + i;
            if (!d[8] && !d[16] && !d[24] && !d[32] && !d[40] && !d[48] && !d[56]) {
                const int dc = d[0] * 4;
                for (int r = 0; r < 8; ++r) o[8 * r] = dc;
                continue;
            }
            int t0, t1, t2, t3, x0, x1, x2, x3;
            idct1d(d[0], d[8], d[16], d[24], d[32], d[40], d[48], d[56], t0, t1, t2, t3, x0, x1, x2, x3);
            x0 += 512; x1 += 512; x2 += 512; x3 += 512;
            o[0] = (x0 + t3) >> 10;
            o[56] = (x0 - t3) >> 10;
            o[8] = (x1 + t2) >> 10;
            o[48] = (x1 - t2) >> 10;
            o[16] = (x2 + t1) >> 10;
            o[40] = (x2 - t1) >> 10;
            o[24] = (x3 + t0) >> 10;
            o[32] = (x3 - t0) >> 10;
        }
        auto clamp8 = [](int x) { return (uint8_t)(x < 0 ? 0 : x > 255 ? 255 : x); };
        for (int r = 0; r < 8; ++r) {  // rows
            const int* s = v + 8 * r;
            uint8_t* o = out + (size_t)r * stride;
            int t0, t1, t2, t3, x0, x1, x2, x3;
            idct1d(s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7], t0, t1, t2, t3, x0, x1, x2, x3);
            // 65536 rounds the >> 17; 128 << 17 is the level shift
            x0 += 65536 + (128 << 17); x1 += 65536 + (128 << 17); x2 += 65536 + (128 << 17); x3 += 65536 + (128 << 17);
            o[0] = clamp8((x0 + t3) >> 17);
            o[7] = clamp8((x0 - t3) >> 17);
            o[1] = clamp8((x1 + t2) >> 17);
            o[6] = clamp8((x1 - t2) >> 17);
            o[2] = clamp8((x2 + t1) >> 17);
            o[5] = clamp8((x2 - t1) >> 17);
            o[3] = clamp8((x3 + t0) >> 17);
            o[4] = clamp8((x3 - t0) >> 17);
        }
    }

    void finish_progressive() {
        int16_t tmp[64];
        for (Component& c : comp)
            for (int by = 0; by < c.bh; ++by)
                for (int bx = 0; bx < c.bw; ++bx) {
                    const int16_t* b = c.coef.data() + ((size_t)by * c.bw + bx) * 64;
                    for (int k = 0; k < 64; ++k) tmp[k] = (int16_t)(b[k] * qt[c.tq][k]);
                    idct_block(tmp, c.pixels.data() + (size_t)by * 8 * c.bw * 8 + (size_t)bx * 8, c.bw * 8);
                }
    }

    bool parse() {
        if (n < 4 || p[0] != 0xFF || p[1] != 0xD8) return fail("not a JPEG");
        pos = 2;
        bool have_frame = false, any_scan = false;
        while (pos < n) {
            int m = byte();
            if (m != 0xFF) continue;  // garbage between segments
            do m = byte(); while (m == 0xFF && pos < n);
            if (m == 0xD9) break;  // EOI
            if (m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;
            const int len = u16() - 2;
            if (len < 0 || pos + (size_t)len > n) return fail("truncated JPEG segment");
            const size_t next = pos + len;
            switch (m) {
                case 0xDB: if (!read_dqt(len)) return false; break;
                case 0xC4: if (!read_dht(len)) return false; break;
                case 0xDD: restart_interval = u16(); break;
                case 0xC0:
                case 0xC1:
                case 0xC2:
                    if (have_frame) return fail("several frames");
                    if (!read_sof(len, m == 0xC2)) return false;
                    have_frame = true;
                    break;
                case 0xC3: case 0xC5: case 0xC6: case 0xC7: case 0xC9: case 0xCA: case 0xCB:
                case 0xCD: case 0xCE: case 0xCF:
                    return fail("lossless, hierarchical and arithmetic-coded JPEGs are not supported");
                case 0xDA:
                    if (!have_frame) return fail("scan before frame");
                    if (!read_sos(len)) return false;
                    if (!decode_scan()) return false;
                    any_scan = true;
                    continue;  // decode_scan left pos at the next marker
                case 0xE0:  // APP0 "JFIF"
                    if (len >= 5 && std::memcmp(p + pos, "JFIF", 5) == 0) jfif = true;
                    break;
                case 0xEE:  // APP14 "Adobe": transform flag at offset 11
                    if (len >= 12 && std::memcmp(p + pos, "Adobe", 5) == 0) adobe_transform = p[pos + 11];
                    break;
                default: break;  // APPn, COM, ...
            }
            pos = next;
        }
        if (!have_frame || !any_scan) return fail("JPEG without image data");
        if (progressive) finish_progressive();
        return true;
    }

    // ---- upsampling + colour conversion ------------------------------------------------------
    // One output row of component c at full resolution (width samples), image row `y`. The ratios are
    // stb's integer ones (hs = hmax / h, vs = vmax / v): 1x1 direct, 1x2 / 2x1 / 2x2 by the triangle
    // filters, anything else nearest (x / hs, y / vs). (Non-integer ratios, which stb mishandles, take
    // the scaled nearest sample here.)
    void upsample_row(const Component& c, int y, std::vector<uint8_t>& out, std::vector<int>& tmp) const {
        const int hs = hmax / c.h, vs = vmax / c.v;
        const int stride = c.bw * 8;
        const int cw = (width * c.h + hmax - 1) / hmax;  // the component's own size in samples
        const int ch = (height * c.v + vmax - 1) / vmax;
        out.resize(width);
        const uint8_t* base = c.pixels.data();
        if (hmax % c.h || vmax % c.v) {
            const uint8_t* row = base + (size_t)std::min(y * c.v / vmax, ch - 1) * stride;
            for (int x = 0; x < width; ++x) out[x] = row[std::min(x * c.h / hmax, cw - 1)];
            return;
        }
        const int sy = std::min(y / vs, ch - 1);
        const uint8_t* near = base + (size_t)sy * stride;
        // the vertical neighbour of the 3:1 filters: the row above for the top output row of a pair, below
        // for the bottom one, clamped at the edges
        const uint8_t* far = base + (size_t)((y & 1) ? std::min(sy + 1, ch - 1) : std::max(sy - 1, 0)) * stride;
        if (hs == 1 && vs == 1) {
            std::memcpy(out.data(), near, width);
        } else if (hs == 1 && vs == 2) {
            for (int x = 0; x < width; ++x) out[x] = (uint8_t)((3 * near[x] + far[x] + 2) >> 2);
        } else if (hs == 2 && vs == 1) {
            if (cw == 1) {
                for (int x = 0; x < width; ++x) out[x] = near[0];
                return;
            }
            tmp.assign(2 * cw, 0);
            tmp[0] = near[0];
            tmp[1] = (near[0] * 3 + near[1] + 2) >> 2;
            int i = 1;
            for (; i < cw - 1; ++i) {
                const int m = 3 * near[i] + 2;
                tmp[2 * i] = (m + near[i - 1]) >> 2;
                tmp[2 * i + 1] = (m + near[i + 1]) >> 2;
            }
            tmp[2 * i] = (near[cw - 2] * 3 + near[cw - 1] + 2) >> 2;  // (stb weights the second-last sample here)
            tmp[2 * i + 1] = near[cw - 1];
            for (int x = 0; x < width; ++x) out[x] = (uint8_t)tmp[x];
        } else if (hs == 2 && vs == 2) {
            tmp.resize(cw);
            for (int x = 0; x < cw; ++x) tmp[x] = 3 * near[x] + far[x];
            if (cw == 1) {
                for (int x = 0; x < width; ++x) out[x] = (uint8_t)((tmp[0] + 2) >> 2);
                return;
            }
            std::vector<int> o(2 * cw);
            o[0] = (tmp[0] + 2) >> 2;
            for (int i = 1; i < cw; ++i) {
                o[2 * i - 1] = (3 * tmp[i - 1] + tmp[i] + 8) >> 4;
                o[2 * i] = (3 * tmp[i] + tmp[i - 1] + 8) >> 4;
            }
            o[2 * cw - 1] = (tmp[cw - 1] + 2) >> 2;
            for (int x = 0; x < width; ++x) out[x] = (uint8_t)o[x];
        } else {
            for (int x = 0; x < width; ++x) out[x] = near[std::min(x / hs, cw - 1)];
        }
    }

    void to_rgba(std::vector<uint8_t>& rgba) const {
        rgba.resize((size_t)width * height * 4);
        const bool rgb = comp.size() == 3 && ((adobe_transform == 0 && !jfif) ||
                                              (comp[0].id == 'R' && comp[1].id == 'G' && comp[2].id == 'B'));
        std::vector<uint8_t> r0, r1, r2;
        std::vector<int> tmp;
        auto fix = [](float x) { return (int)(x * 4096.0f + 0.5f) << 8; };
        const int kr = fix(1.40200f), kg1 = -fix(0.71414f), kg2 = -fix(0.34414f), kb = fix(1.77200f);
        auto clamp8 = [](int x) { return (uint8_t)(x < 0 ? 0 : x > 255 ? 255 : x); };
        for (int y = 0; y < height; ++y) {
            uint8_t* o = rgba.data() + (size_t)y * width * 4;
            upsample_row(comp[0], y, r0, tmp);
            if (comp.size() == 1) {
                for (int x = 0; x < width; ++x) { o[4 * x] = o[4 * x + 1] = o[4 * x + 2] = r0[x]; o[4 * x + 3] = 255; }
                continue;
            }
            upsample_row(comp[1], y, r1, tmp);
            upsample_row(comp[2], y, r2, tmp);
            for (int x = 0; x < width; ++x) {
                if (rgb) {
                    o[4 * x] = r0[x]; o[4 * x + 1] = r1[x]; o[4 * x + 2] = r2[x];
                } else {
                    const int yf = (r0[x] << 20) + (1 << 19);
                    const int cb = r1[x] - 128, cr = r2[x] - 128;
                    o[4 * x + 0] = clamp8((yf + cr * kr) >> 20);
                    o[4 * x + 1] = clamp8((yf + cr * kg1 + ((cb * kg2) & (int)0xffff0000)) >> 20);
                    o[4 * x + 2] = clamp8((yf + cb * kb) >> 20);
                }
                o[4 * x + 3] = 255;
            }
        }
    }
};

}  // namespace

bool IsJpeg(const std::string& bytes) {
    return bytes.size() >= 3 && (uint8_t)bytes[0] == 0xFF && (uint8_t)bytes[1] == 0xD8 && (uint8_t)bytes[2] == 0xFF;
}

bool DecodeJpeg(const std::string& bytes, int& width, int& height, std::vector<uint8_t>& rgba, std::string& error) {
    Decoder d;
    d.p = reinterpret_cast<const uint8_t*>(bytes.data());
    d.n = bytes.size();
    if (!d.parse()) {
        error = d.err.empty() ? "malformed JPEG" : d.err;
        return false;
    }
    d.to_rgba(rgba);
    width = d.width;
    height = d.height;
    return true;
}

}  // namespace Loader
}  // namespace Trident
