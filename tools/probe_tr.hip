// Probe: lane semantics of ds_read_b64_tr_b16 on gfx950 (prints raw (row, col) tags per lane).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s16x4 __attribute__((ext_vector_type(4)));
__global__ void k(int* out) {
  __shared__ __attribute__((aligned(16))) unsigned short lds[16 * 64];
  for (int i = threadIdx.x; i < 16 * 64; i += 64) lds[i] = (unsigned short)(((i / 64) << 8) | (i % 64));
  __syncthreads();
  int l = threadIdx.x, g = l >> 4, fr = l & 15, q4 = fr >> 2, p4 = fr & 3;
  int row = 4 * g + q4, col = 4 * p4;
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(lds + row * 64 + col));
  for (int j = 0; j < 4; ++j) out[l * 4 + j] = (unsigned short)v[j];
}
int main() {
  int* d; hipMalloc(&d, 256 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  int h[256]; hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int j = 0; j < 4; ++j) printf(" (r%d,c%d)", h[l * 4 + j] >> 8, h[l * 4 + j] & 255);
    printf("\n");
  }
  return 0;
}
