// pk_probe — does a packed f32 FMA (v_pk_fma_f32, two lanes' worth of f32
// per instruction) cost one wave's issue slot like v_fma_f32? A wave-bound
// loop of 16 independent-ish FMAs as 16 v_fma_f32, as 8 v_pk_fma_f32 (the same
// flops) and as 16 v_pk_fma_f32, at 1 and 4 waves per SIMD (HIP events).
//   hipcc -O3 --offload-arch=gfx950 -o tools/pk_probe tools/pk_probe.hip && tools/pk_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(64) void k(float* out, int iters) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7};
  const float m = 0.999f, c = 0.001f;
  const f2 mm = {m, m}, cc = {c, c};
  for (int i = 0; i < iters; ++i) {
    if (MODE == 0) {  // 16 v_fma_f32
#define F(x) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(m), "v"(c))
      F(a0); F(a1); F(a2); F(a3); F(a4); F(a5); F(a6); F(a7);
      F(a0); F(a1); F(a2); F(a3); F(a4); F(a5); F(a6); F(a7);
    } else {  // v_pk_fma_f32: 8 (MODE 1) or 16 (MODE 2)
#define P(x) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(mm), "v"(cc))
      P(p0); P(p1); P(p2); P(p3); P(p0); P(p1); P(p2); P(p3);
      if (MODE == 2) { P(p0); P(p1); P(p2); P(p3); P(p0); P(p1); P(p2); P(p3); }
    }
  }
  out[blockIdx.x * 64 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + p0.x + p1.y + p2.x + p3.y;
}

template <int MODE>
float run(int wgs, int iters, float* d) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0), hipEventCreate(&e1);
  k<MODE><<<wgs, 64>>>(d, iters);
  hipEventRecord(e0);
  k<MODE><<<wgs, 64>>>(d, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  float* d;
  hipMalloc(&d, 64 * 4096 * 4 * sizeof(float));
  const int iters = 200000;
  for (int wps : {1, 2, 4}) {
    const int wgs = 1024 * wps;  // 256 CUs x 4 SIMDs x wps waves
    const float t0 = run<0>(wgs, iters, d), t1 = run<1>(wgs, iters, d), t2 = run<2>(wgs, iters, d);
    // cycles per instruction per wave at ~2.4 GHz: ms * 2.4e6 / (iters * instrs)
    printf("waves/SIMD %d: 16 v_fma %.2f ms (%.2f cyc/instr/wave), 8 v_pk_fma %.2f ms (%.2f), 16 v_pk_fma %.2f ms (%.2f)\n",
           wps, t0, t0 * 2.4e6 / (iters * 16.0), t1, t1 * 2.4e6 / (iters * 8.0), t2, t2 * 2.4e6 / (iters * 16.0));
  }
  hipFree(d);
  return 0;
}
