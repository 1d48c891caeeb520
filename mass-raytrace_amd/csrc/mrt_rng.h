// mrt_rng.h — random number streams.
//
// 1) Scene stream: restatement of fastrand 1.4.1's wyrand (Cargo.lock:579-582),
//    the generator behind Num::rand (math.rs:244-246), fastrand::u8(0..3) in
//    BvhNode::new (geom.rs:111) and fastrand::seed(1) (main.rs:86). Published
//    algorithm (fastrand is not vendored under /root/reference, so this is
//    unpinned by any reference test):
//      gen_u64: s += 0xA0761D6478BD642F; t = (u128)s * (s ^ 0xE7037ED1A0B428DB);
//               return lo64(t) ^ hi64(t)
//      f32    : from_bits(0x3F800000 | (gen_u32 >> 9)) - 1.0
//      u8(0..3): Lemire gen_mod_u32(3)
// 2) Path stream: the reference seeds its render threads from the clock, so
//    per-sample randomness is not reproducible there (main.rs:249-265). Here
//    every (pixel, sample) owns a xoroshiro128** stream seeded by splitmix64
//    of (seed, pixel, sample); the f32 mapping is fastrand's, applied to the
//    high 32 bits. Host oracle and GPU share this definition.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define MRT_RNG_HD __host__ __device__ __forceinline__
#else
#define MRT_RNG_HD inline
#endif

namespace mrt {

MRT_RNG_HD float bits_to_unit_f32(uint32_t r) {
  union {
    uint32_t u;
    float f;
  } c;
  c.u = 0x3F800000u | (r >> 9);
  return c.f - 1.0f;
}

// host only (the scene stream never runs on the GPU)
struct WyRand {
  uint64_t state;
  uint64_t gen_u64() {
    uint64_t s = state + 0xA0761D6478BD642FULL;
    state = s;
    unsigned __int128 t = (unsigned __int128)s * (unsigned __int128)(s ^ 0xE7037ED1A0B428DBULL);
    return (uint64_t)t ^ (uint64_t)(t >> 64);
  }
  uint32_t gen_u32() { return (uint32_t)gen_u64(); }
  float f32() { return bits_to_unit_f32(gen_u32()); }
  uint32_t gen_mod_u32(uint32_t n) {
    uint32_t r = gen_u32();
    uint64_t m = (uint64_t)r * (uint64_t)n;
    uint32_t hi = (uint32_t)(m >> 32), lo = (uint32_t)m;
    if (lo < n) {
      uint32_t t = (0u - n) % n;
      while (lo < t) {
        r = gen_u32();
        m = (uint64_t)r * (uint64_t)n;
        hi = (uint32_t)(m >> 32);
        lo = (uint32_t)m;
      }
    }
    return hi;
  }
  // fastrand::u8(0..3)
  uint32_t axis() { return gen_mod_u32(3); }
};

MRT_RNG_HD uint64_t splitmix64_next(uint64_t& x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

MRT_RNG_HD uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

struct PathRng {
  uint64_t s0, s1;
  MRT_RNG_HD uint64_t next() {
    const uint64_t a = s0;
    uint64_t b = s1;
    const uint64_t result = rotl64(a * 5, 7) * 9;
    b ^= a;
    s0 = rotl64(a, 24) ^ b ^ (b << 16);
    s1 = rotl64(b, 37);
    return result;
  }
  MRT_RNG_HD float f32() { return bits_to_unit_f32((uint32_t)(next() >> 32)); }
};

// Stream of sample `sample` of pixel `pixel` (= y*width + x).
MRT_RNG_HD PathRng path_rng(uint64_t seed, uint32_t pixel, uint32_t sample) {
  uint64_t x = seed;
  uint64_t k = splitmix64_next(x);
  x = k ^ (((uint64_t)pixel << 32) | (uint64_t)sample);
  PathRng r;
  r.s0 = splitmix64_next(x);
  r.s1 = splitmix64_next(x);
  if ((r.s0 | r.s1) == 0) r.s1 = 1;
  return r;
}

}  // namespace mrt
