// ImageDecoder.h — PNG (and JPEG, JpegDecoder.cpp) decoding with stb_image's observable semantics, for the texture and skybox
// loaders (TextureLoader.cpp:290-304 loads 2D textures with stbi_load(..., STBI_rgb_alpha) after
// stbi_set_flip_vertically_on_load(true); LoadFromFileList, :773-830, loads cube faces unflipped).
// stb is an un-vendored submodule of the reference, so its PNG path is restated here on zlib:
//   - every critical chunk layout (IHDR / PLTE / tRNS / IDAT / IEND), colour types 0, 2, 3, 4, 6,
//     bit depths 1, 2, 4, 8, 16, the five scanline filters and Adam7 interlacing;
//   - forced 4 channels: grey g -> (g, g, g, 255), grey+alpha -> (g, g, g, a), RGB -> (r, g, b, 255);
//   - 16-bit samples reduced to their high byte (stbi__convert_16_to_8), 1/2/4-bit grey scaled by
//     0xFF / 0x55 / 0x11 (stbi__depth_scale_table), palette indices looked up in PLTE with tRNS alpha;
//   - a tRNS colour key on grey / RGB images gives alpha 0 to matching pixels and 255 elsewhere,
//     compared at the image's own bit depth (stbi__compute_transparency / _16);
//   - chunk CRCs, gamma, sRGB and ICC chunks are ignored, as stb ignores them.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace Trident {
namespace Loader {

// Decodes a PNG held in `bytes` into top-to-bottom RGBA8 rows. Returns false (with `error` set) on
// malformed or unsupported input.
bool DecodePng(const std::string& bytes, int& width, int& height, std::vector<uint8_t>& rgba, std::string& error);

// True when `bytes` starts with the PNG signature.
bool IsPng(const std::string& bytes);

// Decodes a baseline or progressive JPEG (JpegDecoder.cpp: stb_image's JPEG path restated) into
// top-to-bottom RGBA8 rows. Returns false (with `error` set) on malformed or unsupported input.
bool DecodeJpeg(const std::string& bytes, int& width, int& height, std::vector<uint8_t>& rgba, std::string& error);

// True when `bytes` starts with an SOI marker followed by another marker.
bool IsJpeg(const std::string& bytes);

void FlipRowsVertically(std::vector<uint8_t>& rgba, int width, int height);

}  // namespace Loader
}  // namespace Trident
