// LDS-DMA ingest probe: how fast can one block per CU pull bytes into LDS with
// global_load_lds_dwordx4, by access pattern and bytes in flight?
//   mode 0: each instruction = 1 KiB contiguous (one 1 KiB row per wave-instruction)
//   mode 1: each instruction = 16 rows x 64 B (the decode GEMM's A/W tile pattern, row pitch 1 KiB)
//   mode 2: like 1 but 8 rows x 128 B
// The source is `src_kb` KiB (small = L2-resident, large = HBM), each block reads `blk_kb` KiB
// starting at a block-dependent offset, waiting every `inflight_kb` KiB (vmcnt(0) + barrier).
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe_glds.hip -o tools/probe_glds
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

__global__ __launch_bounds__(1024) void ingest(const char* __restrict__ src, long src_bytes, int blk_bytes, int inflight,
                                               int mode, int* sink) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwv = blockDim.x >> 6;
  const long base = ((long)blockIdx.x * 7919 * 1024) & (src_bytes - 1);
  const long b0 = base & ~1023L;
  const int per_group = inflight / (1024 * nwv);  // instructions per wave per group
  for (int g0 = 0; g0 < blk_bytes; g0 += inflight) {
    for (int i = 0; i < per_group; ++i) {
      const int ins = (g0 / 1024) + i * nwv + wave;  // global instruction index (1 KiB each)
      long off;
      if (mode == 0) off = (long)ins * 1024 + lane * 16;
      else if (mode == 1) {  // 16 rows x 64 B: rows of 1 KiB pitch, column block = ins % 16
        const int rb = ins / 16, cb = ins % 16;
        off = (long)(rb * 16 + (lane >> 2)) * 1024 + cb * 64 + (lane & 3) * 16;
      } else {
        const int rb = ins / 8, cb = ins % 8;
        off = (long)(rb * 8 + (lane >> 3)) * 1024 + cb * 128 + (lane & 7) * 16;
      }
      if (mode == 3) continue;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + ((b0 + off) & (src_bytes - 1))),
                                       (__attribute__((address_space(3))) void*)(lds + ((i * nwv + wave) * 1024) % (128 * 1024)),
                                       16, 0, 0);
    }
    if (mode == 3) {
      // register staging, 8 x 16 B per lane in flight, then ds_write_b128
      for (int i0 = 0; i0 < per_group; i0 += 8) {
        uint4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int ins = (g0 / 1024) + (i0 + k) * 4 + wave;
          v[k] = *(const uint4*)(src + ((b0 + (long)ins * 1024 + lane * 16) & (src_bytes - 1)));
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) *(uint4*)(lds + ((((i0 + k) * 4 + wave) * 1024 + lane * 16) & (inflight - 1))) = v[k];
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (threadIdx.x == 0 && lds[5] == 123) sink[blockIdx.x] = 1;
}

int main(int argc, char** argv) {
  const long srcs[] = {512L << 10, 4L << 20, 64L << 20, 1L << 30};
  char* src;
  CK(hipMalloc(&src, 1L << 30));
  CK(hipMemset(src, 1, 1L << 30));
  int* sink;
  CK(hipMalloc(&sink, 4096 * 4));
  CK(hipFuncSetAttribute((const void*)ingest, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024));
  // empty-kernel event overhead
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  printf("%-8s %-5s %-5s %-9s %-6s %10s %12s\n", "srcKB", "mode", "waves", "inflight", "grid", "us", "GB/s/CU");
  const int blk = 1024 * 1024;
  for (long sb : {4L << 20, 64L << 20})
    for (int mode : {0, 1, 2})
      for (int nwv : {16})
        for (int infl : {65536})
          for (int grid : {32, 256, 512}) {
            const int lds = infl;
            for (int rep = 0; rep < 2; ++rep) {
              CK(hipEventRecord(a));
              hipLaunchKernelGGL(ingest, dim3(grid), dim3(nwv * 64), lds, 0, src, sb, blk, infl, mode, sink);
              CK(hipEventRecord(b));
              CK(hipEventSynchronize(b));
            }
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            const double per_cu = (double)grid * blk / std::min(grid, 256) / (ms * 1e-3) / 1e9;
            printf("%-8ld %-5d %-5d %-9d %-6d %10.2f %12.1f\n", sb >> 10, mode, nwv, infl, grid, ms * 1e3, per_cu);
          }
  return 0;
}
