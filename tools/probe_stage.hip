// Chip-level staging ceiling: LDS-DMA (global_load_lds_dwordx4) against register staging
// (global_load_dwordx4 -> VGPRs -> ds_write_b128) and plain register loads, one 512-thread block
// per CU (256 blocks), each wave streaming 1 KiB contiguous per instruction with D instructions in
// flight, from a source of SRC_MB (L2-, MALL- or HBM-resident).  Reports aggregate GB/s.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe_stage.hip -o tools/probe_stage
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// MODE 0: LDS-DMA, wait vmcnt(D - 1) after each issue (D in flight per wave)
// MODE 1: register loads, D in flight, each landed vector written to LDS (ds_write_b128)
// MODE 2: register loads, D in flight, xor-reduced (no LDS)
template <int MODE, int D>
__global__ __launch_bounds__(512) void stream_k(const char* __restrict__ src, long mask, int iters, int* sink) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long base = ((long)blockIdx.x * 7919L * 4096L) & mask;
  auto off = [&](int i) { return (base + ((long)i * 8 + wave) * 1024 + lane * 16) & mask; };
  u32x4 acc = {0u, 0u, 0u, 0u};
  if (MODE == 0) {
    for (int i = 0; i < iters; ++i) {
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + off(i)),
                                       (__attribute__((address_space(3))) void*)(lds + ((i % 16) * 8 + wave) * 1024),
                                       16, 0, 0);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D - 1) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    acc = *(const u32x4*)(lds + threadIdx.x * 16);
  } else {
    u32x4 r[D];
#pragma unroll
    for (int d = 0; d < D; ++d) r[d] = *(const u32x4*)(src + off(d));
    for (int i = D; i < iters; i += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        if (MODE == 1) *(u32x4*)(lds + (((i + d) % 16) * 8 + wave) * 1024 + lane * 16) = r[d];
        else acc ^= r[d];
        r[d] = *(const u32x4*)(src + off(i + d));
      }
    }
#pragma unroll
    for (int d = 0; d < D; ++d) acc ^= r[d];
    if (MODE == 1) acc ^= *(const u32x4*)(lds + threadIdx.x * 16);
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}

template <int MODE, int D>
void run(const char* src, long bytes, int* sink, const char* name) {
  const int grid = 256, iters = 512;  // 512 KiB per wave... 8 waves x 512 x 1 KiB = 4 MiB per block
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL((stream_k<MODE, D>), dim3(grid), dim3(512), 128 * 1024, 0, src, bytes - 1, iters, sink);
  CK(hipEventRecord(a));
  const int reps = 5;
  for (int w = 0; w < reps; ++w) hipLaunchKernelGGL((stream_k<MODE, D>), dim3(grid), dim3(512), 128 * 1024, 0, src, bytes - 1, iters, sink);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  const double moved = (double)grid * 8 * iters * 1024 * reps;
  printf("%-28s src %6ld MiB  D=%2d  %8.1f GB/s  (%.1f GB/s per CU)\n", name, bytes >> 20, D, moved / (ms * 1e-3) / 1e9,
         moved / (ms * 1e-3) / 1e9 / 256);
}

int main() {
  for (auto f : {(const void*)stream_k<0, 4>, (const void*)stream_k<0, 8>, (const void*)stream_k<0, 16>,
                 (const void*)stream_k<1, 4>, (const void*)stream_k<1, 8>, (const void*)stream_k<1, 16>,
                 (const void*)stream_k<2, 8>, (const void*)stream_k<2, 16>})
    CK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024));
  int* sink;
  CK(hipMalloc(&sink, 4));
  for (long mb : {2L, 128L, 2048L}) {
    const long bytes = mb << 20;
    char* src;
    CK(hipMalloc(&src, bytes));
    CK(hipMemset(src, 1, bytes));
    run<0, 4>(src, bytes, sink, "lds-dma");
    run<0, 8>(src, bytes, sink, "lds-dma");
    run<0, 16>(src, bytes, sink, "lds-dma");
    run<1, 4>(src, bytes, sink, "regs -> ds_write");
    run<1, 8>(src, bytes, sink, "regs -> ds_write");
    run<1, 16>(src, bytes, sink, "regs -> ds_write");
    run<2, 8>(src, bytes, sink, "regs only");
    run<2, 16>(src, bytes, sink, "regs only");
    CK(hipFree(src));
  }
  return 0;
}
