// Probe: which MFMA k-slot each (lane, element) of the A and B operands of
// v_mfma_f32_16x16x32_bf16 feeds.  A one-hot at (lane la, element ja) times B one-hot at
// (lane lb, element jb) gives a non-zero C iff both occupy the same k-slot.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void k(int la, int ja, int lb, int jb, float* out) {
  int l = threadIdx.x;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (__bf16)((l == la && j == ja) ? 1.f : 0.f); b[j] = (__bf16)((l == lb && j == jb) ? 1.f : 0.f); }
  f32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}
int main() {
  float* d; (void)hipMalloc(&d, 256 * 4);
  float h[256];
  // fix B at lane lb=0 (col 0), element jb; find which A (lane-group, element) pairs with it
  for (int lb_g = 0; lb_g < 4; ++lb_g)
    for (int jb = 0; jb < 8; ++jb) {
      int lb = lb_g * 16;  // column 0
      printf("B(lane %2d, j %d) pairs with A:", lb, jb);
      for (int ag = 0; ag < 4; ++ag)
        for (int ja = 0; ja < 8; ++ja) {
          int la = ag * 16;  // row 0
          hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, la, ja, lb, jb, d);
          (void)hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
          float s = 0; for (int i = 0; i < 256; ++i) s += h[i];
          if (s != 0) {
            int pos = -1; for (int i = 0; i < 256; ++i) if (h[i] != 0) pos = i;
            printf(" (lane %d, j %d)->C lane %d reg %d", la, ja, pos / 4, pos % 4);
          }
        }
      printf("\n");
    }
  return 0;
}
