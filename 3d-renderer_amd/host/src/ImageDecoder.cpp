// ImageDecoder.cpp — PNG decoding with stb_image's observable semantics (see ImageDecoder.h).
#include "trident/ImageDecoder.h"

#include <zlib.h>

#include <algorithm>
#include <cstring>

namespace Trident {
namespace Loader {

namespace {

uint32_t Be32(const unsigned char* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
uint32_t Be16(const unsigned char* p) { return (uint32_t)p[0] << 8 | p[1]; }

int Channels(int colorType) {
    switch (colorType) {
        case 0: return 1;
        case 2: return 3;
        case 3: return 1;
        case 4: return 2;
        case 6: return 4;
        default: return 0;
    }
}

// stbi__depth_scale_table: grey samples of 1/2/4 bits stretch to 0..255
int DepthScale(int depth) { return depth == 1 ? 0xFF : depth == 2 ? 0x55 : depth == 4 ? 0x11 : 1; }

bool Inflate(const std::string& in, size_t need, std::vector<unsigned char>& out, std::string& error) {
    out.assign(need, 0);
    z_stream zs;
    std::memset(&zs, 0, sizeof zs);
    if (inflateInit(&zs) != Z_OK) {
        error = "zlib init failed";
        return false;
    }
    zs.next_in = reinterpret_cast<Bytef*>(const_cast<char*>(in.data()));
    zs.avail_in = (uInt)in.size();
    zs.next_out = out.data();
    zs.avail_out = (uInt)need;
    const int rc = inflate(&zs, Z_FINISH);
    const size_t got = need - zs.avail_out;
    inflateEnd(&zs);
    // stb only needs enough bytes for the image; a stream that does not end where the image ends
    // (Z_BUF_ERROR with the output full) still decodes
    if (got < need || (rc != Z_STREAM_END && rc != Z_BUF_ERROR && rc != Z_OK)) {
        error = "corrupt or truncated image data";
        return false;
    }
    return true;
}

// In-place PNG scanline unfiltering (filter types 0-4) of `rows` rows of `rowBytes` bytes each, each
// preceded by its filter byte; `dist` = bytes per complete pixel (>= 1).
bool Unfilter(unsigned char* data, size_t rows, size_t rowBytes, size_t dist, std::vector<unsigned char>& outRows,
              std::string& error) {
    outRows.assign(rows * rowBytes, 0);
    std::vector<unsigned char> zero(rowBytes, 0);
    for (size_t y = 0; y < rows; ++y) {
        const unsigned char filter = data[y * (rowBytes + 1)];
        const unsigned char* src = data + y * (rowBytes + 1) + 1;
        unsigned char* cur = outRows.data() + y * rowBytes;
        const unsigned char* prev = y ? outRows.data() + (y - 1) * rowBytes : zero.data();
        for (size_t i = 0; i < rowBytes; ++i) {
            const int a = i >= dist ? cur[i - dist] : 0;
            const int b = prev[i];
            const int c = i >= dist ? prev[i - dist] : 0;
            int v;
            switch (filter) {
                case 0: v = src[i]; break;
                case 1: v = src[i] + a; break;
                case 2: v = src[i] + b; break;
                case 3: v = src[i] + ((a + b) >> 1); break;
                case 4: {  // Paeth
                    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
                    v = src[i] + ((pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c));
                    break;
                }
                default:
                    error = "invalid scanline filter";
                    return false;
            }
            cur[i] = (unsigned char)v;
        }
    }
    return true;
}

uint32_t Sample(const unsigned char* row, size_t index, int depth) {
    if (depth == 8) return row[index];
    if (depth == 16) return Be16(row + 2 * index);
    const size_t bit = index * (size_t)depth;
    return (row[bit >> 3] >> (8 - depth - (int)(bit & 7))) & ((1u << depth) - 1u);
}

}  // namespace

bool IsPng(const std::string& b) {
    static const unsigned char sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
    return b.size() >= 8 && std::memcmp(b.data(), sig, 8) == 0;
}

void FlipRowsVertically(std::vector<uint8_t>& rgba, int w, int h) {
    const size_t row = (size_t)w * 4;
    std::vector<uint8_t> tmp(row);
    for (int y = 0; y < h / 2; ++y) {
        uint8_t* a = rgba.data() + (size_t)y * row;
        uint8_t* b = rgba.data() + (size_t)(h - 1 - y) * row;
        std::memcpy(tmp.data(), a, row);
        std::memcpy(a, b, row);
        std::memcpy(b, tmp.data(), row);
    }
}

bool DecodePng(const std::string& bytes, int& width, int& height, std::vector<uint8_t>& rgba, std::string& error) {
    if (!IsPng(bytes)) {
        error = "not a PNG";
        return false;
    }
    const unsigned char* p = reinterpret_cast<const unsigned char*>(bytes.data());
    size_t pos = 8;
    uint32_t w = 0, h = 0;
    int depth = 0, ctype = -1, interlace = 0;
    bool haveHdr = false, haveEnd = false;
    unsigned char palette[256][4];
    for (auto& e : palette) { e[0] = e[1] = e[2] = 0; e[3] = 255; }
    uint32_t paletteSize = 0;
    bool hasKey = false;
    uint32_t key[3] = {0, 0, 0};
    std::string idat;
    while (!haveEnd) {
        if (pos + 8 > bytes.size()) {
            error = "truncated chunk";
            return false;
        }
        const uint32_t len = Be32(p + pos);
        const std::string type(bytes.data() + pos + 4, 4);
        if ((uint64_t)pos + 12 + len > bytes.size()) {
            error = "truncated chunk";
            return false;
        }
        const unsigned char* d = p + pos + 8;
        if (type == "IHDR") {
            if (len != 13) { error = "bad IHDR"; return false; }
            w = Be32(d);
            h = Be32(d + 4);
            depth = d[8];
            ctype = d[9];
            interlace = d[12];
            if (d[10] != 0 || d[11] != 0 || interlace > 1) { error = "unsupported PNG compression/filter/interlace"; return false; }
            const int ch = Channels(ctype);
            const bool depthOk = depth == 1 || depth == 2 || depth == 4 || depth == 8 || depth == 16;
            if (!ch || !depthOk || (ctype == 3 && depth == 16) || ((ctype == 2 || ctype == 4 || ctype == 6) && depth < 8)) {
                error = "unsupported PNG colour type / bit depth";
                return false;
            }
            if (w == 0 || h == 0 || w > (1u << 24) || h > (1u << 24) || (uint64_t)w * h > (1ull << 28)) {
                error = "bad PNG dimensions";
                return false;
            }
            haveHdr = true;
        } else if (type == "PLTE") {
            if (len % 3 || len / 3 > 256) { error = "bad PLTE"; return false; }
            paletteSize = len / 3;
            for (uint32_t i = 0; i < paletteSize; ++i) {
                palette[i][0] = d[3 * i];
                palette[i][1] = d[3 * i + 1];
                palette[i][2] = d[3 * i + 2];
            }
        } else if (type == "tRNS") {
            if (!haveHdr) { error = "tRNS before IHDR"; return false; }
            if (ctype == 3) {
                if (len > paletteSize) { error = "bad tRNS"; return false; }
                for (uint32_t i = 0; i < len; ++i) palette[i][3] = d[i];
            } else if (ctype == 0 || ctype == 2) {
                const uint32_t n = ctype == 0 ? 1u : 3u;
                if (len != 2 * n) { error = "bad tRNS"; return false; }
                for (uint32_t k = 0; k < n; ++k)  // stb: 8-bit and lower keys compare after depth scaling
                    key[k] = depth == 16 ? Be16(d + 2 * k) : (Be16(d + 2 * k) & 255u) * (uint32_t)DepthScale(depth);
                hasKey = true;
            }
        } else if (type == "IDAT") {
            idat.append(bytes.data() + pos + 8, len);
        } else if (type == "IEND") {
            haveEnd = true;
        } else if (!(type[0] & 0x20)) {  // an unknown critical chunk
            error = "unsupported critical chunk " + type;
            return false;
        }
        pos += 12 + len;  // length, type, data, CRC (not checked, as in stb)
    }
    if (!haveHdr || idat.empty() || (ctype == 3 && paletteSize == 0)) {
        error = "missing IHDR / IDAT / PLTE";
        return false;
    }
    const int ch = Channels(ctype);
    const size_t bitsPerPixel = (size_t)ch * depth;
    const size_t dist = std::max<size_t>(1, bitsPerPixel / 8);
    struct Pass { uint32_t x0, y0, dx, dy; };
    static const Pass adam7[7] = {{0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4}, {0, 2, 2, 4}, {1, 0, 2, 2}, {0, 1, 1, 2}};
    const Pass whole{0, 0, 1, 1};
    const int npass = interlace ? 7 : 1;
    size_t need = 0;
    for (int k = 0; k < npass; ++k) {
        const Pass& ps = interlace ? adam7[k] : whole;
        const size_t pw = w > ps.x0 ? (w - ps.x0 + ps.dx - 1) / ps.dx : 0, ph = h > ps.y0 ? (h - ps.y0 + ps.dy - 1) / ps.dy : 0;
        if (pw && ph) need += ph * (1 + (pw * bitsPerPixel + 7) / 8);
    }
    std::vector<unsigned char> raw;
    if (!Inflate(idat, need, raw, error)) return false;
    rgba.assign((size_t)w * h * 4, 0);
    size_t off = 0;
    std::vector<unsigned char> rows;
    const int scale = DepthScale(depth);
    for (int k = 0; k < npass; ++k) {
        const Pass& ps = interlace ? adam7[k] : whole;
        const size_t pw = w > ps.x0 ? (w - ps.x0 + ps.dx - 1) / ps.dx : 0, ph = h > ps.y0 ? (h - ps.y0 + ps.dy - 1) / ps.dy : 0;
        if (!pw || !ph) continue;
        const size_t rowBytes = (pw * bitsPerPixel + 7) / 8;
        if (!Unfilter(raw.data() + off, ph, rowBytes, dist, rows, error)) return false;
        off += ph * (rowBytes + 1);
        for (size_t y = 0; y < ph; ++y) {
            const unsigned char* row = rows.data() + y * rowBytes;
            for (size_t x = 0; x < pw; ++x) {
                uint8_t* o = rgba.data() + (((size_t)ps.y0 + y * ps.dy) * w + ps.x0 + x * ps.dx) * 4;
                uint32_t s[4] = {0, 0, 0, 0};
                for (int c = 0; c < ch; ++c) s[c] = Sample(row, x * (size_t)ch + c, depth);
                auto to8 = [&](uint32_t v) -> uint8_t { return depth == 16 ? (uint8_t)(v >> 8) : (uint8_t)(v * (uint32_t)scale); };
                switch (ctype) {
                    case 0: {
                        o[0] = o[1] = o[2] = to8(s[0]);
                        const uint32_t cmp = depth == 16 ? s[0] : o[0];
                        o[3] = (hasKey && cmp == key[0]) ? 0 : 255;
                        break;
                    }
                    case 2: {
                        o[0] = to8(s[0]); o[1] = to8(s[1]); o[2] = to8(s[2]);
                        const bool match = depth == 16 ? (s[0] == key[0] && s[1] == key[1] && s[2] == key[2])
                                                       : (o[0] == key[0] && o[1] == key[1] && o[2] == key[2]);
                        o[3] = (hasKey && match) ? 0 : 255;
                        break;
                    }
                    case 3:
                        std::memcpy(o, palette[s[0] & 255], 4);
                        break;
                    case 4:
                        o[0] = o[1] = o[2] = to8(s[0]);
                        o[3] = to8(s[1]);
                        break;
                    default:
                        o[0] = to8(s[0]); o[1] = to8(s[1]); o[2] = to8(s[2]); o[3] = to8(s[3]);
                        break;
                }
            }
        }
    }
    width = (int)w;
    height = (int)h;
    return true;
}

}  // namespace Loader
}  // namespace Trident
