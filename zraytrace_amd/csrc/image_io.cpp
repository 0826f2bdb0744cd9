// image_io.cpp — the reference's image reader and writers over the C ABI.
//
// png_image.zig:19-94 (readFile): decode_png below, zlib instead of libpng.
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
#include <cstdlib>
#include <cstring>
#include <memory>
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

namespace {

uint32_t be32(const uint8_t* p) { return uint32_t(p[0]) << 24 | uint32_t(p[1]) << 16 | uint32_t(p[2]) << 8 | p[3]; }

// PNG filter types 0-4 (PNG spec §9) undone in place on one scanline.
void unfilter_row(uint8_t* row, const uint8_t* prev, size_t n, unsigned bpp, uint8_t type) {
  switch (type) {
    case 0: return;
    case 1:
      for (size_t i = bpp; i < n; ++i) row[i] = uint8_t(row[i] + row[i - bpp]);
      return;
    case 2:
      if (prev)
        for (size_t i = 0; i < n; ++i) row[i] = uint8_t(row[i] + prev[i]);
      return;
    case 3:
      for (size_t i = 0; i < n; ++i) {
        const unsigned a = i >= bpp ? row[i - bpp] : 0, b = prev ? prev[i] : 0;
        row[i] = uint8_t(row[i] + ((a + b) >> 1));
      }
      return;
    case 4:
      for (size_t i = 0; i < n; ++i) {
        const int a = i >= bpp ? row[i - bpp] : 0, b = prev ? prev[i] : 0;
        const int c = (i >= bpp && prev) ? prev[i - bpp] : 0;
        const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
        row[i] = uint8_t(row[i] + (pa <= pb && pa <= pc ? a : pb <= pc ? b : c));
      }
      return;
    default: throw Error(ZRT_E_IO, "BadPngFile: unknown filter type");
  }
}

}  // namespace

// png_image.readFile (png_image.zig:19-94) without libpng: 8-bit RGB or RGBA
// only (other color types / depths are the reference's UnsupportedPngFeature),
// Adam7 de-interlaced as png_read_image does, alpha dropped (png_set_filler),
// rows flipped and each sample stored as f32 sample / 255 (png_image.zig:86-87).
std::unique_ptr<Image> decode_png(const std::string& path, const std::vector<uint8_t>& f) {
  static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  if (f.size() < 8 || std::memcmp(f.data(), sig, 8) != 0) throw Error(ZRT_E_IO, path + ": BadPngFile (signature)");
  uint32_t w = 0, h = 0;
  uint8_t depth = 0, ctype = 0, interlace = 0;
  bool have_ihdr = false, have_iend = false;
  std::vector<uint8_t> idat;
  for (size_t pos = 8; pos + 12 <= f.size();) {
    const uint32_t n = be32(&f[pos]);
    if (n > f.size() - pos - 12) throw Error(ZRT_E_IO, path + ": BadPngFile (truncated chunk)");
    const uint8_t* type = &f[pos + 4];
    const uint8_t* data = &f[pos + 8];
    if (uint32_t(crc32(0L, type, uInt(n + 4))) != be32(data + n))
      throw Error(ZRT_E_IO, path + ": BadPngFile (chunk CRC)");
    if (std::memcmp(type, "IHDR", 4) == 0) {
      if (n != 13) throw Error(ZRT_E_IO, path + ": BadPngFile (IHDR)");
      w = be32(data);
      h = be32(data + 4);
      depth = data[8];
      ctype = data[9];
      if (data[10] != 0 || data[11] != 0 || data[12] > 1) throw Error(ZRT_E_IO, path + ": BadPngFile (IHDR methods)");
      interlace = data[12];
      have_ihdr = true;
    } else if (std::memcmp(type, "IDAT", 4) == 0) {
      idat.insert(idat.end(), data, data + n);
    } else if (std::memcmp(type, "IEND", 4) == 0) {
      have_iend = true;
      break;
    }
    pos += size_t(n) + 12;
  }
  if (!have_ihdr || !have_iend || w == 0 || h == 0) throw Error(ZRT_E_IO, path + ": BadPngFile");
  // png_image.zig:44-51
  if (ctype != 2 && ctype != 6)
    throw Error(ZRT_E_UNSUPPORTED, path + ": UnsupportedPngFeature (color type " + std::to_string(ctype) + ")");
  if (depth != 8)
    throw Error(ZRT_E_UNSUPPORTED, path + ": UnsupportedPngFeature (bit depth " + std::to_string(depth) + ")");
  if (uint64_t(w) * h > (1ull << 30)) throw Error(ZRT_E_UNSUPPORTED, path + ": image too large");
  const unsigned bpp = ctype == 6 ? 4 : 3;
  // Adam7 passes {x0, y0, dx, dy}; a non-interlaced image is one pass
  static const uint32_t adam7[7][4] = {{0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4},
                                       {0, 2, 2, 4}, {1, 0, 2, 2}, {0, 1, 1, 2}};
  static const uint32_t single[1][4] = {{0, 0, 1, 1}};
  const int n_pass = interlace ? 7 : 1;
  const uint32_t(*passes)[4] = interlace ? adam7 : single;
  size_t raw_size = 0;
  for (int p = 0; p < n_pass; ++p) {
    const uint32_t x0 = passes[p][0], y0 = passes[p][1], dx = passes[p][2], dy = passes[p][3];
    if (w <= x0 || h <= y0) continue;  // an empty pass has no scanlines, not even filter bytes
    const size_t pw = (w - x0 + dx - 1) / dx, ph = (h - y0 + dy - 1) / dy;
    raw_size += ph * (1 + pw * bpp);
  }
  std::vector<uint8_t> raw(raw_size + 1);  // + 1: a stream longer than the image is an error
  z_stream zs;
  std::memset(&zs, 0, sizeof(zs));
  if (inflateInit(&zs) != Z_OK) throw Error(ZRT_E_NOMEM, "OutOfMemory (inflate)");
  zs.next_in = idat.data();
  zs.avail_in = uInt(idat.size());
  zs.next_out = raw.data();
  zs.avail_out = uInt(raw.size());
  const int zrc = inflate(&zs, Z_FINISH);
  const size_t produced = raw.size() - zs.avail_out;
  inflateEnd(&zs);
  if (zrc != Z_STREAM_END || produced != raw_size) throw Error(ZRT_E_IO, path + ": BadPngFile (IDAT stream)");
  std::vector<uint8_t> px(size_t(w) * h * bpp);
  size_t at = 0;
  for (int p = 0; p < n_pass; ++p) {
    const uint32_t x0 = passes[p][0], y0 = passes[p][1], dx = passes[p][2], dy = passes[p][3];
    if (w <= x0 || h <= y0) continue;
    const size_t pw = (w - x0 + dx - 1) / dx, ph = (h - y0 + dy - 1) / dy, stride = pw * bpp;
    const uint8_t* prev = nullptr;  // the first scanline of a pass has none
    for (size_t r = 0; r < ph; ++r) {
      uint8_t* row = &raw[at + 1];
      unfilter_row(row, prev, stride, bpp, raw[at]);
      for (size_t i = 0; i < pw; ++i)
        std::memcpy(&px[((y0 + r * dy) * size_t(w) + x0 + i * dx) * bpp], row + i * bpp, bpp);
      prev = row;
      at += 1 + stride;
    }
  }
  auto img = Image::init(w, h);
  for (uint32_t y = 0; y < h; ++y) {
    for (uint32_t x = 0; x < w; ++x) {
      const uint8_t* s = &px[(size_t(y) * w + x) * bpp];
      float* o = &img->pixels[((size_t(h) - y - 1) * w + x) * 3];  // image_offset = (height - y - 1) * width + x
      o[0] = float(s[0]) / 255.0f;  // @intToFloat(f32, px0) / 0xff
      o[1] = float(s[1]) / 255.0f;
      o[2] = float(s[2]) / 255.0f;
    }
  }
  return img;
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

int zrt_image_read_png(const char* path, uint32_t* width, uint32_t* height, float** out_pixels) {
  if (!path || !width || !height || !out_pixels) return zrt::fail(ZRT_E_INVALID, "null argument");
  *out_pixels = nullptr;
  try {
    std::unique_ptr<zrt::Image> img = zrt::readImageFile(path);
    float* p = static_cast<float*>(std::malloc(sizeof(float) * img->pixels.size()));
    if (!p) return zrt::fail(ZRT_E_NOMEM, "OutOfMemory");
    std::memcpy(p, img->pixels.data(), sizeof(float) * img->pixels.size());
    *width = img->width;
    *height = img->height;
    *out_pixels = p;
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
