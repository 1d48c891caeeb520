// buf_check — do bounded buffer loads (make_buffer_rsrc + raw_buffer_load_b128,
// the form path.h uses) return the same words as plain global loads on gfx950?
//   hipcc -O3 --offload-arch=gfx950 -o tools/buf_check tools/buf_check.hip && tools/buf_check
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef uint32_t u4v __attribute__((ext_vector_type(4)));
struct In {
  const uint4* p;
  uint32_t n;
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(nullptr, (short)0, 0, 0);
};
__device__ __forceinline__ uint4 bl(const In& in, uint32_t i) {
  const u4v v = __builtin_amdgcn_raw_buffer_load_b128(in.r, i * 16u, 0, 0);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__global__ void k(const uint4* p, uint32_t n, uint32_t* bad, uint32_t* oob) {
  const In in{p, n, __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(p), (short)0, (int)(n * 16u), 0x00020000)};
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t i = (t * 2654435761u) % n;
  const uint4 a = bl(in, i), b = p[i];
  if (a.x != b.x || a.y != b.y || a.z != b.z || a.w != b.w) atomicAdd(bad, 1u);
  const uint4 c = bl(in, n + (t & 1023));  // past the range: zeros
  if (c.x | c.y | c.z | c.w) atomicAdd(oob, 1u);
}
int main() {
  const uint32_t n = 1u << 20;
  std::vector<uint32_t> h(4 * (size_t)n);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (uint32_t)(i * 747796405u + 1u);
  uint4* d;
  uint32_t* c;
  (void)hipMalloc(&d, h.size() * 4 + (1 << 20));
  (void)hipMalloc(&c, 8);
  (void)hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemset(c, 0, 8);
  hipLaunchKernelGGL(k, dim3(4096), dim3(256), 0, 0, d, n, c, c + 1);
  uint32_t r[2];
  (void)hipMemcpy(r, c, 8, hipMemcpyDeviceToHost);
  printf("buffer vs global mismatches: %u of %u; nonzero past range: %u\n", r[0], 4096u * 256u, r[1]);
  return r[0] != 0;
}
