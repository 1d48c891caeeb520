// ta_probe — cost of gathered vector loads on gfx950, to choose k_trace's
// record format: wave load instructions per CU-cycle for loads of 1-4 dwords
// per lane, 64 / 32 / 16 active lanes, random vs wave-uniform vs 4-way
// shared addresses, from an L1-sized and an L2-sized table.
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/ta_probe tools/ta_probe.hip && /tmp/ta_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u2 __attribute__((ext_vector_type(2)));
typedef uint32_t u3 __attribute__((ext_vector_type(3)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));

template <int W>
__device__ __forceinline__ uint32_t ld(const uint32_t* p) {
  if constexpr (W == 1) return *p;
  if constexpr (W == 2) { u2 v = *reinterpret_cast<const u2*>(p); return v.x ^ v.y; }
  if constexpr (W == 3) { u3 v = *reinterpret_cast<const u3*>(p); return v.x ^ v.y ^ v.z; }
  if constexpr (W == 4) { u4 v = *reinterpret_cast<const u4*>(p); return (v.x ^ v.y) ^ (v.z ^ v.w); }
}

// PAT 0: every lane its own random 16-B slot; 1: one slot per wave; 2: 4 slots per wave (16 lanes each);
// 3: two loads per lane to the two halves of one random 32-B record (the k_trace box step)
template <int W, int PAT>
__global__ __launch_bounds__(256) void k_probe(const uint32_t* tab, uint32_t mask, int iters, int active,
                                               uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63;
  uint32_t h = (blockIdx.x * 256u + threadIdx.x) * 2654435761u + 12345u;
  uint32_t acc = 0;
  if (lane < (uint32_t)active) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        h = h * 1664525u + 1013904223u;
        uint32_t key = h >> 8;
        if (PAT == 1) {
          key = __builtin_amdgcn_readfirstlane(key);
          asm volatile("" : "+v"(key));  // keep the uniform address in a VGPR: vector loads
        }
        if (PAT == 2) key = __shfl(key, lane & 48u, 64);
        if (PAT == 3) {
          const uint32_t* p = tab + ((key & mask) & ~1u) * 4u;
          acc += ld<W>(p) ^ ld<W>(p + 4);
        } else {
          acc += ld<W>(tab + (key & mask) * 4u);
        }
      }
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <int W, int PAT>
static void run(const uint32_t* d_tab, uint32_t slots, int active, int cus, uint32_t* d_out, const char* tname) {
  const int blocks = cus * 8, iters = 2000;  // 8 x 256 threads per CU = 8 waves per SIMD
  hipLaunchKernelGGL((k_probe<W, PAT>), dim3(blocks), dim3(256), 0, 0, d_tab, slots - 1, 50, active, d_out);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL((k_probe<W, PAT>), dim3(blocks), dim3(256), 0, 0, d_tab, slots - 1, iters, active, d_out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double waves = blocks * 4.0, instr = waves * iters * 4 * (PAT == 3 ? 2 : 1);
  const double per_cu_ns = instr / cus / (ms * 1e6);  // wave load instructions per CU per ns
  const double lanes_gb = instr * active * W * 4 / (ms * 1e-3) / 1e9;
  printf("%-4s W=%d pat=%d active=%2d  %8.3f ms  %6.3f instr/CU/ns  (%5.1f cyc/instr @2.4GHz)  %8.0f GB/s lane data\n",
         tname, W, PAT, active, ms, per_cu_ns, 2.4 / per_cu_ns, lanes_gb);
  hipEventDestroy(a);
  hipEventDestroy(b);
}

template <int PAT>
static void sweep(const uint32_t* d, uint32_t slots, int cus, uint32_t* o, const char* tn) {
  for (int act : {64, 32, 16}) {
    run<1, PAT>(d, slots, act, cus, o, tn);
    run<2, PAT>(d, slots, act, cus, o, tn);
    run<3, PAT>(d, slots, act, cus, o, tn);
    run<4, PAT>(d, slots, act, cus, o, tn);
  }
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  printf("%s, %d CUs\n", p.gcnArchName, cus);
  const uint32_t big = 1u << 16;  // 1 MiB of 16-B slots
  std::vector<uint32_t> h(big * 4);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (uint32_t)(i * 2654435761u);
  uint32_t *d, *o;
  hipMalloc(&d, h.size() * 4);
  hipMalloc(&o, 64);
  hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  for (uint32_t slots : {1024u, big}) {
    const char* tn = slots == 1024u ? "16K" : "1M";
    sweep<0>(d, slots, cus, o, tn);
    sweep<1>(d, slots, cus, o, tn);
    sweep<2>(d, slots, cus, o, tn);
    run<4, 3>(d, slots, 64, cus, o, tn);
    run<3, 3>(d, slots, 64, cus, o, tn);
  }
  hipFree(d);
  hipFree(o);
  return 0;
}
