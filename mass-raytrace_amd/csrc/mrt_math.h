// mrt_math.h — f32 vector/matrix arithmetic shared by the C++ host and the
// gfx950 kernels. Every operation is written in the reference's evaluation
// order so host and device agree bit for bit (compile with
// -ffp-contract=off, no fast-math; device division/sqrt are the correctly
// rounded IEEE forms):
//   V3 ops        /root/reference/src/math/generic.rs:7-43,197-312
//   dot           generic.rs:8-10   (x*x' + y*y') + z*z'
//   cross         generic.rs:12-18
//   unit/length   math.rs:250-260   v / sqrt(dot(v,v)), three divides
//   reflect       math.rs:297-299   v - (n*dot)*2
//   refract       math.rs:301-306
//   near_zero     math.rs:293-295
//   M4 transform  generic.rs:105-124 ((c0*x + c1*y) + c2*z) + c3*w
//   M4 mul        generic.rs:126-159 (transpose + V4 dot, left to right)
#pragma once
#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define MRT_HD __host__ __device__ __forceinline__
#else
#define MRT_HD inline
#endif

namespace mrt {

struct V2 {
  float x, y;
};
struct V3 {
  float x, y, z;
};
struct V4 {
  float x, y, z, w;
};

// RN(1/x), the value `1.0f / x` has under -fhip-fp32-correctly-rounded-
// divide-sqrt: on the device v_rcp_f32 (within an ulp) and one FMA Newton
// step for |x| in [2^-126, 2^126) — checked equal for every one of the 2^32
// floats (tools/rcp_check.hip) — else the IEEE division (zero, infinities,
// NaN, subnormals, the top binade). 3 instructions instead of ~11.
MRT_HD float rcp_cr(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  const float ax = fabsf(x);
  if (ax >= 0x1p-126f && ax < 0x1p126f) {
    const float r = __builtin_amdgcn_rcpf(x);
    return fmaf(fmaf(-x, r, 1.0f), r, r);
  }
#endif
  return 1.0f / x;
}
MRT_HD V2 v2(float x, float y) { return V2{x, y}; }
MRT_HD V3 v3(float x, float y, float z) { return V3{x, y, z}; }
MRT_HD V3 fill3(float f) { return V3{f, f, f}; }
MRT_HD V4 v4(float x, float y, float z, float w) { return V4{x, y, z, w}; }

MRT_HD V3 operator+(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
MRT_HD V3 operator-(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
MRT_HD V3 operator*(V3 a, V3 b) { return V3{a.x * b.x, a.y * b.y, a.z * b.z}; }
MRT_HD V3 operator/(V3 a, V3 b) { return V3{a.x / b.x, a.y / b.y, a.z / b.z}; }
MRT_HD V3 operator*(V3 a, float s) { return V3{a.x * s, a.y * s, a.z * s}; }
MRT_HD V3 operator/(V3 a, float s) { return V3{a.x / s, a.y / s, a.z / s}; }
MRT_HD V3 operator-(V3 a) { return V3{-a.x, -a.y, -a.z}; }
// f32 / V3 (generic.rs:221-229): per component s / v
MRT_HD V3 sdiv(float s, V3 a) { return V3{s / a.x, s / a.y, s / a.z}; }

MRT_HD V2 operator+(V2 a, V2 b) { return V2{a.x + b.x, a.y + b.y}; }
MRT_HD V2 operator-(V2 a, V2 b) { return V2{a.x - b.x, a.y - b.y}; }
MRT_HD V2 operator*(V2 a, float s) { return V2{a.x * s, a.y * s}; }

MRT_HD V4 operator+(V4 a, V4 b) { return V4{a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }
MRT_HD V4 operator-(V4 a, V4 b) { return V4{a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w}; }
MRT_HD V4 operator*(V4 a, float s) { return V4{a.x * s, a.y * s, a.z * s, a.w * s}; }

MRT_HD float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
MRT_HD V3 cross(V3 a, V3 b) {
  return V3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
MRT_HD float length_squared(V3 a) { return dot(a, a); }
MRT_HD float length(V3 a) { return sqrtf(length_squared(a)); }
MRT_HD V3 unit(V3 a) { return a / length(a); }
// Rust f32::min/max ignore a NaN operand, as fminf/fmaxf do.
MRT_HD V3 vmin(V3 a, V3 b) { return V3{fminf(a.x, b.x), fminf(a.y, b.y), fminf(a.z, b.z)}; }
MRT_HD V3 vmax(V3 a, V3 b) { return V3{fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z)}; }
MRT_HD bool near_zero(V3 a) {
  return fabsf(a.x) <= 0.00001f && fabsf(a.y) <= 0.00001f && fabsf(a.z) <= 0.00001f;
}
MRT_HD V3 reflect(V3 v, V3 n) { return v - ((n * dot(v, n)) * 2.0f); }
MRT_HD V3 refract(V3 v, V3 n, float etai_over_etat) {
  float cos_theta = fminf(dot(-v, n), 1.0f);
  V3 r_out_perp = (v + n * cos_theta) * etai_over_etat;
  V3 r_out_parallel = n * -sqrtf(fabsf(1.0f - length_squared(r_out_perp)));
  return r_out_perp + r_out_parallel;
}

// Column-major 4x4 (generic.rs:71-77); only the xyz rows of each column are
// needed for transform_point/vector, but the w row is kept for M4 products.
struct M4 {
  V4 c0, c1, c2, c3;
};
MRT_HD float dot4(V4 a, V4 b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }
MRT_HD V3 transform(const M4& m, V3 p, float w) {
  V4 vx = m.c0 * p.x, vy = m.c1 * p.y, vz = m.c2 * p.z, vw = m.c3 * w;
  V4 v = ((vx + vy) + vz) + vw;
  return V3{v.x, v.y, v.z};
}
MRT_HD V3 transform_point(const M4& m, V3 p) { return transform(m, p, 1.0f); }
MRT_HD V3 transform_vector(const M4& m, V3 p) { return transform(m, p, 0.0f); }

inline M4 m4_transpose(const M4& m) {
  return M4{V4{m.c0.x, m.c1.x, m.c2.x, m.c3.x}, V4{m.c0.y, m.c1.y, m.c2.y, m.c3.y},
            V4{m.c0.z, m.c1.z, m.c2.z, m.c3.z}, V4{m.c0.w, m.c1.w, m.c2.w, m.c3.w}};
}
inline M4 m4_mul(const M4& a, const M4& b) {
  M4 m = m4_transpose(a);
  return M4{V4{dot4(m.c0, b.c0), dot4(m.c1, b.c0), dot4(m.c2, b.c0), dot4(m.c3, b.c0)},
            V4{dot4(m.c0, b.c1), dot4(m.c1, b.c1), dot4(m.c2, b.c1), dot4(m.c3, b.c1)},
            V4{dot4(m.c0, b.c2), dot4(m.c1, b.c2), dot4(m.c2, b.c2), dot4(m.c3, b.c2)},
            V4{dot4(m.c0, b.c3), dot4(m.c1, b.c3), dot4(m.c2, b.c3), dot4(m.c3, b.c3)}};
}
// constructors: math.rs:357-406 (angles in turns: (a*PI)*2 then sin_cos)
constexpr float kPi = 3.14159265358979323846f;
// glibc sinf/cosf behind out-of-line wrappers (defined in host/world.cpp) so
// the compiler cannot fuse them into sincosf (math.rs:367 calls sin_cos)
float host_sinf(float x);
float host_cosf(float x);
float host_tanf(float x);
inline M4 m4_translation(V3 t) {
  return M4{V4{1, 0, 0, 0}, V4{0, 1, 0, 0}, V4{0, 0, 1, 0}, V4{t.x, t.y, t.z, 1}};
}
inline M4 m4_rotate_x(float a) {
  float r = (a * kPi) * 2.0f, s = host_sinf(r), c = host_cosf(r);
  return M4{V4{1, 0, 0, 0}, V4{0, c, s, 0}, V4{0, -s, c, 0}, V4{0, 0, 0, 1}};
}
inline M4 m4_rotate_y(float a) {
  float r = (a * kPi) * 2.0f, s = host_sinf(r), c = host_cosf(r);
  return M4{V4{c, 0, s, 0}, V4{0, 1, 0, 0}, V4{-s, 0, c, 0}, V4{0, 0, 0, 1}};
}
inline M4 m4_rotate_z(float a) {
  float r = (a * kPi) * 2.0f, s = host_sinf(r), c = host_cosf(r);
  return M4{V4{c, -s, 0, 0}, V4{s, c, 0, 0}, V4{0, 0, 1, 0}, V4{0, 0, 0, 1}};
}
inline M4 m4_scale(V3 s) {
  return M4{V4{s.x, 0, 0, 0}, V4{0, s.y, 0, 0}, V4{0, 0, s.z, 0}, V4{0, 0, 0, 1}};
}

}  // namespace mrt
