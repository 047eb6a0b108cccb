// Probe: how fast can 256 one-per-CU blocks pull their weight tiles in at kernel start?
// (the decode-step kernels' prologue pattern; tools/probe_ingest.sh)
//   mode 0: 16 waves x 16 global_load_dwordx4 into VGPRs, each instruction 16 rows x 64 B (dec_ffn pattern)
//   mode 1: the same bytes, each wave instruction 1 KiB contiguous
//   mode 2: the same bytes by LDS-DMA (global_load_lds_dwordx4, 1 KiB per instruction) into a 128 KiB ring
//   mode 3: mode 0 but every block reads slice 0 (all blocks share one 256 KiB tile)
//   mode 4: mode 0 with 4 loads per wave in flight at a time (4 rounds)
// usage: ./probe_ingest [kb_per_block=256] [blocks=256]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int MODE, int NLOAD>
__global__ __launch_bounds__(1024) void probe(const unsigned char* __restrict__ w, long slice_bytes, int nslices,
                                              unsigned* out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = MODE == 3 ? 0 : blockIdx.x % nslices;
  const unsigned char* base = w + (long)j * slice_bytes;
  const long per_wave = slice_bytes / 16;  // bytes per wave
  constexpr int nload = NLOAD;
  u32x4 acc = {0, 0, 0, 0};
  if (MODE == 2) {
    for (int i = 0; i < nload; ++i) {
      const unsigned char* src = base + wave * per_wave + i * 1024 + lane * 16;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(smem + ((wave * nload + i) % 128) * 1024),
                                       16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    acc = *(const u32x4*)(smem + threadIdx.x * 16 % 131072);
  } else {
    constexpr int rounds = (MODE == 4 && NLOAD >= 4) ? 4 : 1;
    constexpr int per_round = NLOAD / rounds;
    u32x4 r[per_round];
    const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
    for (int rd = 0; rd < rounds; ++rd) {
#pragma unroll
      for (int i = 0; i < per_round; ++i) {
        const int li = rd * per_round + i;
        const unsigned char* src;
        if (MODE == 1) src = base + wave * per_wave + li * 1024 + lane * 16;
        else src = base + wave * per_wave + (long)fr * (per_wave / 16) + li * 64 + fq * 16;  // 16 rows x 64 B
        r[i] = *(const u32x4*)src;
      }
#pragma unroll
      for (int i = 0; i < per_round; ++i) acc += r[i];
    }
  }
  if (acc[0] == 0x12345678u) out[blockIdx.x] = acc[1];
}

int main(int argc, char** argv) {
  const long kb = argc > 1 ? atol(argv[1]) : 256;
  const int blocks = argc > 2 ? atoi(argv[2]) : 256;
  const long slice = kb * 1024;
  const int nslices = 16;
  unsigned char* w;
  unsigned* out;
  CHK(hipMalloc(&w, slice * nslices));
  CHK(hipMemset(w, 1, slice * nslices));
  CHK(hipMalloc(&out, blocks * 4));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  const int nl = (int)(slice / 16 / 1024);
  for (int mode = 0; mode < 5; ++mode) {
    auto launch = [&]() {
#define P(M, N) hipLaunchKernelGGL((probe<M, N>), dim3(blocks), dim3(1024), M == 2 ? 131072 : 0, 0, w, slice, nslices, out)
#define PN(M) do { if (nl == 16) P(M, 16); else if (nl == 8) P(M, 8); else if (nl == 4) P(M, 4); else P(M, 1); } while (0)
      switch (mode) { case 0: PN(0); break; case 1: PN(1); break; case 2: PN(2); break; case 3: PN(3); break; default: PN(4); }
    };
    const int reps = 40;
    for (int it = 0; it < 5; ++it) launch();
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(a, 0));
    for (int it = 0; it < reps; ++it) launch();
    CHK(hipGetLastError());
    CHK(hipEventRecord(b, 0));
    CHK(hipEventSynchronize(b));
    float ms;
    CHK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / reps;
    const double bytes = (double)slice * blocks;
    printf("mode %d  %4ld KiB/block x %d blocks: %7.2f us per launch (back to back) -> %6.2f TB/s, %6.1f GB/s per block\n",
           mode, kb, blocks, us, bytes / (us * 1e-6) / 1e12, slice / (us * 1e-6) / 1e9);
  }
  return 0;
}
