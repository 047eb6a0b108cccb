// probe: device-side icap_drop_hash against the host build of the same function (tools/, measurement)
#include <cstdio>
#include "../image_caption_amd/csrc/common.h"
__global__ void k(const uint32_t* in, uint32_t* out, int n) {
  int i = threadIdx.x;
  if (i < n) out[i] = icap_drop_hash(in[6 * i], in[6 * i + 1], in[6 * i + 2], in[6 * i + 3], in[6 * i + 4], in[6 * i + 5]);
}
int main() {
  const uint32_t t[4][6] = {{4242, 4, 1, 1, 0, 43}, {4242, 4, 1, 3, 0, 158}, {4242, 6, 4, 6, 0, 436}, {4242, 3, 0, 1, 0, 1442}};
  uint32_t *din, *dout, out[4];
  hipMalloc(&din, sizeof(t));
  hipMalloc(&dout, sizeof(out));
  hipMemcpy(din, t, sizeof(t), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, din, dout, 4);
  hipMemcpy(out, dout, sizeof(out), hipMemcpyDeviceToHost);
  for (int i = 0; i < 4; ++i)
    printf("device %u host %u\n", out[i], icap_drop_hash(t[i][0], t[i][1], t[i][2], t[i][3], t[i][4], t[i][5]));
  return 0;
}
