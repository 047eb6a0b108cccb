// Debug harness for enc_attention: V = identity so O = P; checks P vs a CPU softmax.
#include "../image_caption_amd/csrc/attention.hip"
#include <cstdio>
#include <cstring>
#include <cmath>
#include <vector>
static uint16_t tobf(float f) { uint32_t u; memcpy(&u, &f, 4); return (uint16_t)((u + 0x7FFF + ((u >> 16) & 1)) >> 16); }
static float frbf(uint16_t h) { uint32_t u = (uint32_t)h << 16; float f; memcpy(&f, &u, 4); return f; }
int main() {
  for (int mode = 0; mode < 2; ++mode) {
    const int B = 1, N = 7, H = 1, D = 64, ld = 3 * D;
    std::vector<uint16_t> qkv(B * N * ld, 0);
    srand(1);
    for (int n = 0; n < N; ++n)
      for (int d = 0; d < D; ++d) {
        float q = mode == 0 ? 0.f : (rand() % 17 - 8) / 4.f, k = mode == 0 ? 0.f : (rand() % 17 - 8) / 4.f;
        qkv[n * ld + d] = tobf(q);
        qkv[n * ld + D + d] = tobf(k);
        qkv[n * ld + 2 * D + d] = tobf(n == d ? 1.f : 0.f);
      }
    uint16_t *dq, *dout;
    (void)hipMalloc(&dq, qkv.size() * 2);
    (void)hipMalloc(&dout, B * N * D * 2);
    (void)hipMemcpy(dq, qkv.data(), qkv.size() * 2, hipMemcpyHostToDevice);
    (void)hipMemset(dout, 0, B * N * D * 2);
    hipError_t e = launch_enc_attention(dq, ld, 0, B, N, H, 0.125f, dout, D, 0, 1, 0);
    (void)hipDeviceSynchronize();
    std::vector<uint16_t> out(B * N * D);
    (void)hipMemcpy(out.data(), dout, out.size() * 2, hipMemcpyDeviceToHost);
    printf("mode %d launch=%d\n", mode, (int)e);
    double maxerr = 0;
    for (int q = 0; q < N; ++q) {
      double s[64], m = -1e30, l = 0;
      for (int k = 0; k < N; ++k) {
        double acc = 0;
        for (int d = 0; d < D; ++d) acc += frbf(qkv[q * ld + d]) * frbf(qkv[k * ld + D + d]);
        s[k] = acc / 8; m = fmax(m, s[k]);
      }
      for (int k = 0; k < N; ++k) { s[k] = exp(s[k] - m); l += s[k]; }
      printf(" q%d got:", q);
      for (int d = 0; d < 10; ++d) printf(" %.4f", frbf(out[q * D + d]));
      printf("\n    ref:");
      for (int d = 0; d < 10; ++d) printf(" %.4f", d < N ? s[d] / l : 0.0);
      printf("\n");
      for (int d = 0; d < D; ++d) maxerr = fmax(maxerr, fabs(frbf(out[q * D + d]) - (d < N ? s[d] / l : 0.0)));
    }
    printf("mode %d maxerr %g\n", mode, maxerr);
  }
  return 0;
}
