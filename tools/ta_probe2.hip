// ta_probe2 — cost per wave instruction of one 16-B gather by addressing form
// (64-bit VGPR address, SGPR base + 32-bit VGPR offset, buffer resource +
// offset) and of ds_read_b128, for random and 4-way shared addresses from an
// L1-sized table: which form k_trace's record loads should take.
//   hipcc -O3 --offload-arch=gfx950 -o tools/ta_probe2 tools/ta_probe2.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

// FORM 0: global v[addr64]; 1: global voff, s[base]; 2: buffer_load offen; 3: ds_read_b128
// 4: global_load_dwordx4 + global_load_dwordx4 offset:16 on one 64-bit address (the box step)
template <int FORM, int PAT>
__global__ __launch_bounds__(256) void k_probe(const uint32_t* tab, uint32_t mask, int iters, uint32_t* out) {
  __shared__ u4 lds[1024];
  const uint32_t lane = threadIdx.x & 63;
  if (FORM == 3) {
    for (uint32_t k = threadIdx.x; k < 1024; k += 256) lds[k] = reinterpret_cast<const u4*>(tab)[k];
    __syncthreads();
  }
  uint32_t h = (blockIdx.x * 256u + threadIdx.x) * 2654435761u + 12345u;
  u4 acc = {0, 0, 0, 0};
  typedef int i4 __attribute__((ext_vector_type(4)));
  const uint64_t base = (uint64_t)(uintptr_t)tab;
  const i4 rsrc = {__builtin_amdgcn_readfirstlane((int)(uint32_t)base), __builtin_amdgcn_readfirstlane((int)(uint32_t)(base >> 32)),
                   0x7FFFFFFF, 0x00020000};  // no stride, num_records, raw dword format (CDNA3/4)
  for (int it = 0; it < iters; ++it) {
    u4 r0, r1, r2, r3;
    uint32_t off[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      h = h * 1664525u + 1013904223u;
      uint32_t key = h >> 8;
      if (PAT == 2) key = __shfl(key, lane & 48u, 64);
      off[k] = (key & mask) * 16u;
    }
    if (FORM == 0 || FORM == 4) {
      const char* b = reinterpret_cast<const char*>(tab);
      const char *p0 = b + off[0], *p1 = b + off[1], *p2 = b + off[2], *p3 = b + off[3];
      if (FORM == 0) {
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r0) : "v"(p0));
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r1) : "v"(p1));
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r2) : "v"(p2));
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r3) : "v"(p3));
      } else {
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r0) : "v"(p0));
        asm volatile("global_load_dwordx4 %0, %1, off offset:16" : "=v"(r1) : "v"(p0));
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r2) : "v"(p1));
        asm volatile("global_load_dwordx4 %0, %1, off offset:16" : "=v"(r3) : "v"(p1));
      }
    } else if (FORM == 1) {
      asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(r0) : "v"(off[0]), "s"(tab));
      asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(r1) : "v"(off[1]), "s"(tab));
      asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(r2) : "v"(off[2]), "s"(tab));
      asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(r3) : "v"(off[3]), "s"(tab));
    } else if (FORM == 2) {
      asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(r0) : "v"(off[0]), "s"(rsrc));
      asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(r1) : "v"(off[1]), "s"(rsrc));
      asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(r2) : "v"(off[2]), "s"(rsrc));
      asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(r3) : "v"(off[3]), "s"(rsrc));
    } else {
      const uint32_t lb = (uint32_t)(uintptr_t)lds;
      asm volatile("ds_read_b128 %0, %1" : "=v"(r0) : "v"(lb + off[0]));
      asm volatile("ds_read_b128 %0, %1" : "=v"(r1) : "v"(lb + off[1]));
      asm volatile("ds_read_b128 %0, %1" : "=v"(r2) : "v"(lb + off[2]));
      asm volatile("ds_read_b128 %0, %1" : "=v"(r3) : "v"(lb + off[3]));
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    asm volatile("v_xor_b32 %0, %0, %1" : "+v"(acc.x) : "v"(r0.x ^ r1.y));
    asm volatile("v_xor_b32 %0, %0, %1" : "+v"(acc.y) : "v"(r2.z ^ r3.w));
  }
  if ((acc.x ^ acc.y) == 0x12345678u) out[0] = acc.x;
}

template <int FORM, int PAT>
static void run(const uint32_t* d_tab, uint32_t slots, int cus, uint32_t* d_out, const char* name) {
  const int blocks = cus * 8, iters = 2000;
  hipLaunchKernelGGL((k_probe<FORM, PAT>), dim3(blocks), dim3(256), 0, 0, d_tab, slots - 1, 50, d_out);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL((k_probe<FORM, PAT>), dim3(blocks), dim3(256), 0, 0, d_tab, slots - 1, iters, d_out);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  const double instr = blocks * 4.0 * iters * 4;
  const double per_cu_ns = instr / cus / (ms * 1e6);
  printf("%-34s pat=%d  %8.3f ms  %5.1f cyc/instr/CU @2.4GHz\n", name, PAT, ms, 2.4 / per_cu_ns);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const uint32_t slots = 1024;  // 16 KiB
  std::vector<uint32_t> h(slots * 4);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (uint32_t)(i * 2654435761u);
  uint32_t *d, *o;
  (void)hipMalloc(&d, h.size() * 4);
  (void)hipMalloc(&o, 64);
  (void)hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  run<0, 0>(d, slots, cus, o, "global x4 vaddr64");
  run<1, 0>(d, slots, cus, o, "global x4 saddr+voff32");
  run<2, 0>(d, slots, cus, o, "buffer x4 offen");
  run<3, 0>(d, slots, cus, o, "ds_read_b128");
  run<4, 0>(d, slots, cus, o, "global x4 pair (+16) vaddr64");
  run<0, 2>(d, slots, cus, o, "global x4 vaddr64");
  run<1, 2>(d, slots, cus, o, "global x4 saddr+voff32");
  run<2, 2>(d, slots, cus, o, "buffer x4 offen");
  run<3, 2>(d, slots, cus, o, "ds_read_b128");
  run<4, 2>(d, slots, cus, o, "global x4 pair (+16) vaddr64");
  (void)hipFree(d);
  (void)hipFree(o);
  return 0;
}
