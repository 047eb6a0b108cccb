// ResNet-101 trunk helpers (GridFeatureEncoder.cnn, grid:51 = torchvision resnet101 children[:-2]).
// Activations are NHWC bf16 hi/lo planes ([B][H][W][C], lo plane at +lo); every convolution is an
// MFMA GEMM over rows = output pixels (gemm.hip, BatchNorm as the fp32 scale/shift epilogue, the
// residual added from planes before the ReLU).  These kernels produce the GEMM A operands that are
// not the activation itself: the 7x7/2 stem patches from the NCHW fp32 image, the 3x3 patches
// (stride 1 or 2, pad 1) in (kh, kw, c) order = the packed weight order, the stride-2 subsample
// of a 1x1 downsample, and the 3x3/2 max-pool.
#include "common.h"
#include "kernels.h"

namespace {

// img (B,3,224,224) fp32 -> rows (B*112*112) x Kp, k = (kh*7 + kw)*3 + c for k < 147, 0 beyond
__global__ void stem_im2col_kernel(const float* __restrict__ img, int B, int HW, int OH, int Kp, bf16_t* out, long lo,
                                   int nsplit) {
  const long total = (long)B * OH * OH * Kp;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int k = (int)(i % Kp);
    const long r = i / Kp;
    const int ow = (int)(r % OH), oh = (int)((r / OH) % OH), b = (int)(r / ((long)OH * OH));
    float v = 0.f;
    if (k < 147) {
      const int c = k % 3, kw = (k / 3) % 7, kh = k / 21;
      const int y = oh * 2 - 3 + kh, x = ow * 2 - 3 + kw;
      if (y >= 0 && y < HW && x >= 0 && x < HW) v = img[(((long)b * 3 + c) * HW + y) * HW + x];
    }
    bf16_t hv, lv;
    split_bf(v, hv, lv);
    out[i] = hv;
    if (nsplit == 2) out[i + lo] = lv;
  }
}

// planes [B][H][W][C] -> rows (B*OH*OW) x 9C, k = (kh*3 + kw)*C + c; 8 channels per thread
__global__ void im2col3_kernel(const bf16_t* __restrict__ x, long xlo, int B, int H, int W, int C, int stride, int OH,
                               int OW, bf16_t* out, long lo, int nsplit) {
  const int C8 = C / 8;
  const long total = (long)B * OH * OW * 9 * C8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % C8);
    const long t = i / C8;
    const int tap = (int)(t % 9);
    const long r = t / 9;
    const int ow = (int)(r % OW), oh = (int)((r / OW) % OH), b = (int)(r / ((long)OH * OW));
    const int y = oh * stride - 1 + tap / 3, xx = ow * stride - 1 + tap % 3;
    u32x4 h = {0, 0, 0, 0}, l = {0, 0, 0, 0};
    if (y >= 0 && y < H && xx >= 0 && xx < W) {
      const long src = (((long)b * H + y) * W + xx) * C + c8 * 8;
      h = *(const u32x4*)(x + src);
      if (nsplit == 2) l = *(const u32x4*)(x + src + xlo);
    }
    const long dst = r * 9 * C + (long)tap * C + c8 * 8;
    *(u32x4*)(out + dst) = h;
    if (nsplit == 2) *(u32x4*)(out + dst + lo) = l;
  }
}

// planes [B][H][W][C] -> [B][H/2][W/2][C] (every other pixel: the 1x1 stride-2 downsample input)
__global__ void subsample2_kernel(const bf16_t* __restrict__ x, long xlo, int B, int H, int W, int C, bf16_t* out,
                                  long lo, int nsplit) {
  const int C8 = C / 8, OH = (H + 1) / 2, OW = (W + 1) / 2;
  const long total = (long)B * OH * OW * C8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % C8);
    const long r = i / C8;
    const int ow = (int)(r % OW), oh = (int)((r / OW) % OH), b = (int)(r / ((long)OH * OW));
    const long src = (((long)b * H + 2 * oh) * W + 2 * ow) * C + c8 * 8;
    const long dst = r * C + c8 * 8;
    *(u32x4*)(out + dst) = *(const u32x4*)(x + src);
    if (nsplit == 2) *(u32x4*)(out + dst + lo) = *(const u32x4*)(x + src + xlo);
  }
}

// 3x3 / stride 2 / pad 1 max-pool on planes (the value is hi + lo; -inf padding like torch)
__global__ void maxpool3s2_kernel(const bf16_t* __restrict__ x, long xlo, int B, int H, int W, int C, int OH, int OW,
                                  bf16_t* out, long lo, int nsplit) {
  const long total = (long)B * OH * OW * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long r = i / C;
    const int ow = (int)(r % OW), oh = (int)((r / OW) % OH), b = (int)(r / ((long)OH * OW));
    float m = -INFINITY;
    for (int dy = 0; dy < 3; ++dy) {
      const int y = oh * 2 - 1 + dy;
      if (y < 0 || y >= H) continue;
      for (int dx = 0; dx < 3; ++dx) {
        const int xx = ow * 2 - 1 + dx;
        if (xx < 0 || xx >= W) continue;
        const long src = (((long)b * H + y) * W + xx) * C + c;
        float v = bf2f(x[src]);
        if (nsplit == 2) v += bf2f(x[src + xlo]);
        m = fmaxf(m, v);
      }
    }
    bf16_t hv, lv;
    split_bf(m, hv, lv);
    out[i] = hv;
    if (nsplit == 2) out[i + lo] = lv;
  }
}

int grid_for(long n) { return (int)std::min<long>((n + 255) / 256, 65536); }

}  // namespace

hipError_t launch_stem_im2col(const float* img, int B, int HW, int OH, int Kp, bf16_t* out, long lo, int nsplit,
                              hipStream_t s) {
  if (Kp < 147 || Kp % 32) return hipErrorInvalidValue;
  hipLaunchKernelGGL(stem_im2col_kernel, dim3(grid_for((long)B * OH * OH * Kp)), dim3(256), 0, s, img, B, HW, OH,
                     Kp, out, lo, nsplit);
  return hipGetLastError();
}

hipError_t launch_im2col3(const bf16_t* x, long xlo, int B, int H, int W, int C, int stride, int OH, int OW,
                          bf16_t* out, long lo, int nsplit, hipStream_t s) {
  if (C % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(im2col3_kernel, dim3(grid_for((long)B * OH * OW * 9 * (C / 8))), dim3(256), 0, s, x, xlo, B, H,
                     W, C, stride, OH, OW, out, lo, nsplit);
  return hipGetLastError();
}

hipError_t launch_subsample2(const bf16_t* x, long xlo, int B, int H, int W, int C, bf16_t* out, long lo, int nsplit,
                             hipStream_t s) {
  if (C % 8) return hipErrorInvalidValue;
  const long n = (long)B * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8);
  hipLaunchKernelGGL(subsample2_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, xlo, B, H, W, C, out, lo, nsplit);
  return hipGetLastError();
}

hipError_t launch_maxpool3s2(const bf16_t* x, long xlo, int B, int H, int W, int C, int OH, int OW, bf16_t* out,
                             long lo, int nsplit, hipStream_t s) {
  hipLaunchKernelGGL(maxpool3s2_kernel, dim3(grid_for((long)B * OH * OW * C)), dim3(256), 0, s, x, xlo, B, H, W, C,
                     OH, OW, out, lo, nsplit);
  return hipGetLastError();
}

namespace {

// torch conv weight [Cout][Cin][kh][kw] fp32 -> [Cout][Kp] bf16 in (kh, kw, c) order, zero for k >= K
__global__ void pack_conv_kernel(const float* __restrict__ w, int cout, int cin, int k, int Kp, bf16_t* out) {
  const long total = (long)cout * Kp;
  const int K = cin * k * k;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int kk = (int)(i % Kp);
    const long o = i / Kp;
    float v = 0.f;
    if (kk < K) {
      const int c = kk % cin, tap = kk / cin, kh = tap / k, kw = tap % k;
      v = w[((o * cin + c) * k + kh) * k + kw];
    }
    out[i] = f2bf(v);
  }
}

// eval BatchNorm as y = x * scale + shift: scale = gamma / sqrt(var + eps), shift = beta - mean * scale
__global__ void bn_fold_kernel(const float* g, const float* b, const float* mean, const float* var, int C, float eps,
                               float* scale, float* shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float sc = g[c] / sqrtf(var[c] + eps);
  scale[c] = sc;
  shift[c] = b[c] - mean[c] * sc;
}

}  // namespace

hipError_t launch_pack_conv(const float* w, int cout, int cin, int k, int Kp, bf16_t* out, hipStream_t s) {
  if (Kp < cin * k * k) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pack_conv_kernel, dim3(grid_for((long)cout * Kp)), dim3(256), 0, s, w, cout, cin, k, Kp, out);
  return hipGetLastError();
}

hipError_t launch_bn_fold(const float* g, const float* b, const float* mean, const float* var, int C, float eps,
                          float* scale, float* shift, hipStream_t s) {
  hipLaunchKernelGGL(bn_fold_kernel, dim3((C + 255) / 256), dim3(256), 0, s, g, b, mean, var, C, eps, scale, shift);
  return hipGetLastError();
}
