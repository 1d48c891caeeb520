// display.cpp — see display.h.
#include "display.h"

#include <math.h>
#include <stdio.h>
#include <string.h>
#include <zlib.h>

#include <mutex>
#include <vector>

namespace mrt {

namespace {
// Rust f32::min / f32::max (the non-NaN operand wins) and `as u8` (saturating,
// NaN -> 0, truncation toward zero)
float rmin(float a, float b) { return a != a ? b : (b != b ? a : (a < b ? a : b)); }
float rmax(float a, float b) { return a != a ? b : (b != b ? a : (a > b ? a : b)); }
uint8_t as_u8(float v) {
  if (!(v > 0.0f)) return 0;
  if (v >= 255.0f) return 255;
  return (uint8_t)v;
}
}  // namespace

uint8_t gamma_byte_host(float x) {
  volatile float g = 1.0f / 2.2f;  // f32 division, as `1.0 / 2.2` on f32 in the reference
  return as_u8(rmax(rmin(powf(x, g), 1.0f), 0.0f) * 255.0f);
}

const std::array<uint32_t, 256>& gamma_thresholds() {
  static std::array<uint32_t, 256> t{};
  static std::once_flag once;
  std::call_once(once, [] {
    t[0] = 0;
    for (int k = 1; k < 256; ++k) {
      uint32_t lo = 0, hi = 0x3F800000u;  // byte(1.0) == 255
      while (lo < hi) {
        uint32_t mid = lo + (hi - lo) / 2;
        float x;
        memcpy(&x, &mid, 4);
        if (gamma_byte_host(x) >= k)
          hi = mid;
        else
          lo = mid + 1;
      }
      t[k] = lo;
    }
  });
  return t;
}

namespace {
void put32(std::vector<uint8_t>& v, uint32_t x) {
  v.push_back((uint8_t)(x >> 24)), v.push_back((uint8_t)(x >> 16)), v.push_back((uint8_t)(x >> 8)),
      v.push_back((uint8_t)x);
}
void chunk(std::vector<uint8_t>& out, const char* type, const std::vector<uint8_t>& data) {
  put32(out, (uint32_t)data.size());
  size_t start = out.size();
  out.insert(out.end(), type, type + 4);
  out.insert(out.end(), data.begin(), data.end());
  uLong crc = crc32(0L, Z_NULL, 0);
  crc = crc32(crc, out.data() + start, (uInt)(out.size() - start));
  put32(out, (uint32_t)crc);
}
}  // namespace

bool write_png_rgb8(const std::string& path, uint32_t w, uint32_t h, const uint8_t* rgb, std::string& err) {
  if (w == 0 || h == 0 || !rgb) {
    err = "empty image";
    return false;
  }
  std::vector<uint8_t> raw;
  raw.reserve((size_t)h * (3 * (size_t)w + 1));
  for (uint32_t y = 0; y < h; ++y) {
    raw.push_back(0);  // filter: none
    raw.insert(raw.end(), rgb + (size_t)y * w * 3, rgb + ((size_t)y + 1) * w * 3);
  }
  uLongf zlen = compressBound((uLong)raw.size());
  std::vector<uint8_t> z(zlen);
  if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK) {
    err = "zlib compress failed";
    return false;
  }
  z.resize(zlen);
  std::vector<uint8_t> png = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
  std::vector<uint8_t> ihdr;
  put32(ihdr, w);
  put32(ihdr, h);
  ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});  // 8-bit, truecolour, deflate, no filter, no interlace
  chunk(png, "IHDR", ihdr);
  chunk(png, "IDAT", z);
  chunk(png, "IEND", {});
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) {
    err = "cannot open " + path;
    return false;
  }
  bool ok = fwrite(png.data(), 1, png.size(), f) == png.size();
  ok = (fclose(f) == 0) && ok;
  if (!ok) err = "write failed: " + path;
  return ok;
}

}  // namespace mrt
