// image_io.cpp — the reference's image writers over the C ABI.
//
// png_image.zig:96-148 (writeFile): 8-bit RGB, rows written top first (the
// framebuffer's row 0 is the bottom: image_offset = (height - y - 1) * width + x),
// each channel @floatToInt(u8, std.math.clamp(255.999 * c, 0, 0xff)).
// ppm_image.zig (writeFile): plain P3 text with the same row order and
// @floatToInt(u32, value * 255.999) clamped to [0, 255].
//
// The PNG stream is written with zlib (filter 0 on every row) rather than
// libpng; the decoded pixels are the reference's bytes, the compressed bytes
// need not be libpng's.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include <zlib.h>

#include "zrt.hpp"

namespace zrt {

namespace {

// std.math.min / max are `x < y ? x : y` / `x > y ? x : y`; clamp = max(lower, min(val, upper)).
inline float clamp_z(float v, float lo, float hi) {
  const float m = v < hi ? v : hi;
  return lo > m ? lo : m;
}

// png_image.zig:136-138
inline uint8_t png_channel(float c) {
  const float v = clamp_z(255.999f * c, 0.0f, 255.0f);
  return uint8_t(v);  // @floatToInt truncates toward zero; v is in [0, 255]
}

// ppm_image.zig:11-15.  @floatToInt(u32, x) is illegal for x < 0, x >= 2^32 or
// NaN (a safety panic in Debug, undefined in ReleaseFast); here those map to
// the nearest end of [0, 255].
inline uint32_t ppm_channel(float value) {
  const float x = value * 255.999f;
  if (!(x >= 0.0f)) return 0;
  if (x >= 4294967296.0f) return 255;
  const uint32_t v = uint32_t(x);
  return v > 255u ? 255u : v;
}

void put_be32(std::vector<uint8_t>& out, uint32_t v) {
  out.push_back(uint8_t(v >> 24));
  out.push_back(uint8_t(v >> 16));
  out.push_back(uint8_t(v >> 8));
  out.push_back(uint8_t(v));
}

void put_chunk(std::vector<uint8_t>& out, const char type[4], const uint8_t* data, size_t n) {
  put_be32(out, uint32_t(n));
  const size_t at = out.size();
  out.insert(out.end(), type, type + 4);
  if (n) out.insert(out.end(), data, data + n);
  const uLong crc = crc32(0L, out.data() + at, uInt(n + 4));
  put_be32(out, uint32_t(crc));
}

void write_all(const char* path, const void* data, size_t n) {
  FILE* fp = std::fopen(path, "wb");
  if (!fp) throw Error(ZRT_E_IO, std::string("Can't open file ") + path);  // png_image.zig:99
  const size_t w = std::fwrite(data, 1, n, fp);
  const int rc = std::fclose(fp);
  if (w != n || rc != 0) throw Error(ZRT_E_IO, std::string("short write to ") + path);
}

void check_image(const char* path, const float* rgb, uint32_t width, uint32_t height) {
  if (!path || !rgb) throw Error(ZRT_E_INVALID, "null argument");
  if (width == 0 || height == 0) throw Error(ZRT_E_INVALID, "empty image");
}

}  // namespace

std::vector<uint8_t> encode_png(const float* rgb, uint32_t width, uint32_t height) {
  const size_t row = size_t(width) * 3 + 1;  // filter byte + RGB
  std::vector<uint8_t> raw(row * height);
  for (uint32_t y = 0; y < height; ++y) {
    uint8_t* dst = raw.data() + y * row;
    dst[0] = 0;  // filter type None
    const float* src = rgb + (size_t(height - y - 1) * width) * 3;
    for (size_t i = 0; i < size_t(width) * 3; ++i) dst[1 + i] = png_channel(src[i]);
  }
  uLongf zlen = compressBound(uLong(raw.size()));
  std::vector<uint8_t> z(zlen);
  if (compress2(z.data(), &zlen, raw.data(), uLong(raw.size()), Z_DEFAULT_COMPRESSION) != Z_OK)
    throw Error(ZRT_E_NOMEM, "OutOfMemory (deflate)");
  std::vector<uint8_t> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  std::vector<uint8_t> ihdr;
  put_be32(ihdr, width);
  put_be32(ihdr, height);
  ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});  // 8 bit, PNG_COLOR_TYPE_RGB, default methods, no interlace
  put_chunk(out, "IHDR", ihdr.data(), ihdr.size());
  put_chunk(out, "IDAT", z.data(), zlen);
  put_chunk(out, "IEND", nullptr, 0);
  return out;
}

std::string encode_ppm(const char* filename, const float* rgb, uint32_t width, uint32_t height) {
  std::string s;
  s.reserve(size_t(width) * height * 13 + 256);
  s += "P3\n# filename: ";
  s += filename;
  s += "\n# The P3 = colors are in ASCII\n# Image width and height\n";
  s += std::to_string(width) + " " + std::to_string(height) + "\n# Max color value\n255\n# RGB triplets\n";
  char buf[32];
  for (uint32_t y = 0; y < height; ++y) {
    const float* src = rgb + (size_t(height - y - 1) * width) * 3;
    for (uint32_t x = 0; x < width; ++x) {  // "{d: >3} {d: >3} {d: >3}  "
      std::snprintf(buf, sizeof(buf), "%3u %3u %3u  ", ppm_channel(src[3 * x]), ppm_channel(src[3 * x + 1]),
                    ppm_channel(src[3 * x + 2]));
      s += buf;
    }
    s += "\n";
  }
  return s;
}

}  // namespace zrt

extern "C" {

int zrt_image_write_png(const char* path, const float* rgb, uint32_t width, uint32_t height) {
  try {
    zrt::check_image(path, rgb, width, height);
    const std::vector<uint8_t> png = zrt::encode_png(rgb, width, height);
    zrt::write_all(path, png.data(), png.size());
    return ZRT_OK;
  } catch (const zrt::Error& e) {
    return zrt::fail(e.code, e.what());
  } catch (const std::bad_alloc&) {
    return zrt::fail(ZRT_E_NOMEM, "OutOfMemory");
  }
}

int zrt_image_write_ppm(const char* path, const float* rgb, uint32_t width, uint32_t height) {
  try {
    zrt::check_image(path, rgb, width, height);
    const std::string ppm = zrt::encode_ppm(path, rgb, width, height);
    zrt::write_all(path, ppm.data(), ppm.size());
    return ZRT_OK;
  } catch (const zrt::Error& e) {
    return zrt::fail(e.code, e.what());
  } catch (const std::bad_alloc&) {
    return zrt::fail(ZRT_E_NOMEM, "OutOfMemory");
  }
}

}  // extern "C"
