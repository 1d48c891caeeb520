// display.h — host side of Image::to_rgb_bytes / dump (main.rs:640-722,
// 760-783): the gamma byte table and the PNG writer.
#pragma once
#include <stdint.h>

#include <array>
#include <string>

namespace mrt {

// Default mode maps a component x = sum/passes to
//   ((x.powf(1/2.2)).min(1.0).max(0.0) * 255.0) as u8.
// For x in [0, 1] that byte is non-decreasing in x, so it is fully described
// by 255 thresholds: t[k] = bits of the smallest x with byte >= k (t[0] = 0).
// They are derived here from the host libm powf — the function the
// reference calls — so the device's table lookup reproduces the reference's
// byte for every x (checked exhaustively over all 2^30 floats in [0, 1] by
// tests/test_tonemap.py). x < 0 or NaN -> 255 (powf gives NaN; Rust's min
// returns 1.0), x >= 1 -> 255.
const std::array<uint32_t, 256>& gamma_thresholds();
uint8_t gamma_byte_host(float x);

// 8-bit RGB PNG, rows as given (top row first). Returns false with `err`.
bool write_png_rgb8(const std::string& path, uint32_t w, uint32_t h, const uint8_t* rgb, std::string& err);

}  // namespace mrt
