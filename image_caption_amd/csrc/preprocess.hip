// On-GPU image preprocessing: decoded RGB uint8 images of any size ->
// the normalised (B, 3, S, S) fp32 batch the encoders take, bit-identical to the reference's
// torchvision-on-PIL eval transforms (Resize(256) + CenterCrop(224), or Resize((224, 224));
// ToTensor; Normalize(ImageNet mean/std)), i.e. to Pillow's 8-bit bilinear resampler:
//   weights  - per output coordinate, triangle filter of support max(scale, 1) around
//              center = (xx + 0.5) * scale, normalised by their double sum, then Q22 fixed point
//              int(w * 2^22 + 0.5); computed here on the fly in double, in Pillow's operation
//              order and with FP contraction off, so every integer weight matches;
//   passes   - horizontal first into a uint8 intermediate (acc = 2^21 + sum(px * k),
//              clamp(acc >> 22)), then vertical; a pass whose size is unchanged is a copy.
// Only the source rows / output columns the crop keeps are resampled.  The CPU restatement
// (oracle/preprocess.py) is pinned against Pillow itself (tests/test_preprocess.py).
//
// Per-image geometry (int32 x 8, computed by the host wrapper image_caption_amd/preprocess.py):
//   in_h, in_w, rs_h, rs_w (resized size), top, left (crop origin in the resized image),
//   y0, nrows (source rows the vertical pass reads).
#include "common.h"
#include "kernels.h"

#include <algorithm>

#pragma clang fp contract(off)

namespace {

constexpr int PREC = 22;

struct Taps {
  int xmin, n;
  double center, ss, ww;
};

// Pillow precompute_coeffs for one output coordinate (bilinear filter, support 1)
__device__ Taps taps_for(int in_size, int out_size, int xx) {
  const double scale = (double)in_size / (double)out_size;
  const double filterscale = scale > 1.0 ? scale : 1.0;
  const double support = 1.0 * filterscale;
  Taps t;
  t.center = (xx + 0.5) * scale;
  t.ss = 1.0 / filterscale;
  int xmin = (int)(t.center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(t.center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  t.xmin = xmin;
  t.n = xmax - xmin;
  double ww = 0.0;
  for (int x = 0; x < t.n; ++x) {
    double a = (x + xmin - t.center + 0.5) * t.ss;
    if (a < 0.0) a = -a;
    ww += a < 1.0 ? 1.0 - a : 0.0;
  }
  t.ww = ww;
  return t;
}

__device__ __forceinline__ int weight_q22(const Taps& t, int x) {
  double a = (x + t.xmin - t.center + 0.5) * t.ss;
  if (a < 0.0) a = -a;
  double w = a < 1.0 ? 1.0 - a : 0.0;
  if (t.ww != 0.0) w /= t.ww;
  return (int)(0.5 + w * (double)(1 << PREC));
}

__device__ __forceinline__ int clip8(int acc) {
  const int v = acc >> PREC;
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}

// tmp[b][r][x][4]: source row y0 + r, resized column left + x (horizontal pass or copy)
__global__ void prep_horizontal_kernel(const uint8_t* __restrict__ px, const int64_t* __restrict__ offs,
                                       const int32_t* __restrict__ geom, int S, int max_rows, uint8_t* tmp) {
  const int b = blockIdx.y;
  const int32_t* g = geom + b * 8;
  const int in_h = g[0], in_w = g[1], rs_w = g[3], left = g[5], y0 = g[6], nrows = g[7];
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int r = t / S, x = t - r * S;
  if (r >= nrows) return;
  const int y = y0 + r;
  const uint8_t* row = px + offs[b] + (long)y * in_w * 3;
  int c0, c1, c2;
  if (rs_w == in_w) {
    const uint8_t* p = row + (left + x) * 3;
    c0 = p[0];
    c1 = p[1];
    c2 = p[2];
  } else {
    const Taps tp = taps_for(in_w, rs_w, left + x);
    int s0 = 1 << (PREC - 1), s1 = s0, s2 = s0;
    for (int k = 0; k < tp.n; ++k) {
      const int w = weight_q22(tp, k);
      const uint8_t* p = row + (tp.xmin + k) * 3;
      s0 += p[0] * w;
      s1 += p[1] * w;
      s2 += p[2] * w;
    }
    c0 = clip8(s0);
    c1 = clip8(s1);
    c2 = clip8(s2);
  }
  (void)in_h;
  *(uint32_t*)(tmp + (((long)b * max_rows + r) * S + x) * 4) = (uint32_t)c0 | ((uint32_t)c1 << 8) | ((uint32_t)c2 << 16);
}

// out[b][c][y][x] = (u8 / 255 - mean[c]) / std[c], u8 = vertical pass (or copy) at resized row top + y
__global__ void prep_vertical_kernel(const uint8_t* __restrict__ tmp, const int32_t* __restrict__ geom, int S,
                                     int max_rows, float* out) {
  const int b = blockIdx.y;
  const int32_t* g = geom + b * 8;
  const int in_h = g[0], rs_h = g[2], top = g[4], y0 = g[6];
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= S * S) return;
  const int y = t / S, x = t - y * S;
  const uint8_t* col = tmp + ((long)b * max_rows * S + x) * 4;
  const long rstride = (long)S * 4;
  int c[3];
  if (rs_h == in_h) {
    const uint8_t* p = col + (top + y - y0) * rstride;
    c[0] = p[0];
    c[1] = p[1];
    c[2] = p[2];
  } else {
    const Taps tp = taps_for(in_h, rs_h, top + y);
    int s0 = 1 << (PREC - 1), s1 = s0, s2 = s0;
    for (int k = 0; k < tp.n; ++k) {
      const int w = weight_q22(tp, k);
      const uint8_t* p = col + (tp.xmin + k - y0) * rstride;
      s0 += p[0] * w;
      s1 += p[1] * w;
      s2 += p[2] * w;
    }
    c[0] = clip8(s0);
    c[1] = clip8(s1);
    c[2] = clip8(s2);
  }
  const float mean[3] = {0.485f, 0.456f, 0.406f}, stdv[3] = {0.229f, 0.224f, 0.225f};
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    const float v = (float)c[ch] / 255.0f;
    out[(((long)b * 3 + ch) * S + y) * S + x] = (v - mean[ch]) / stdv[ch];
  }
}

}  // namespace

hipError_t launch_preprocess(const uint8_t* px, const int64_t* offs, const int32_t* geom, int B, int S, int max_rows,
                             uint8_t* tmp, float* out, hipStream_t s) {
  if (B <= 0 || S <= 0 || max_rows <= 0 || B > 65535) return hipErrorInvalidValue;
  const long h_threads = (long)max_rows * S;
  hipLaunchKernelGGL(prep_horizontal_kernel, dim3((unsigned)((h_threads + 255) / 256), B), dim3(256), 0, s, px, offs,
                     geom, S, max_rows, tmp);
  hipLaunchKernelGGL(prep_vertical_kernel, dim3((S * S + 255) / 256, B), dim3(256), 0, s, tmp, geom, S, max_rows,
                     out);
  return hipGetLastError();
}
